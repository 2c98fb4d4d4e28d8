"""GPU parity of the HIP kernels, called through the C ABI, against the reference's golden vectors
and the C oracle.  Tolerances (north star): RGB within 1e-4, sigma within 1e-5 (relative to
max(1, |sigma|)); integer/index work (hash gathers, SH, ray geometry) bit-exact."""
import numpy as np
import pytest
import torch

import goldens as G
from oracle import oracle as O

pytestmark = pytest.mark.gpu

DEV = "cuda"
RGB_TOL = 1e-4
SIGMA_TOL = 1e-5


def _t(a):
    return torch.from_numpy(np.ascontiguousarray(a)).to(DEV)


def _ops():
    from adaptive_city_nerf_amd import ops
    return ops


def _spec(d, k, mask, prefix="w:", weights=None):
    ops = _ops()
    sc = G.scene()["masks"][mask]
    w = weights if weights is not None else G.expert_weights(d, k, prefix)
    tab = _t(G.table(int(d["table_seeds"][k]), float(d["table_scale"])))
    res = O.level_resolutions(16, 16, 4096)
    mlp = {key: _t(v) for key, v in w.items() if key in ops.MLP_SHAPES}
    return ops.ExpertSpec(tab, res.tolist(), 20, 1, sc["mins"][k], d[f"w:submodules.{k}.aabb_extent"].tolist(), mlp)


def _oracle_expert(d, k, mask, prefix="w:", weights=None):
    sc = G.scene()["masks"][mask]
    w = weights if weights is not None else G.expert_weights(d, k, prefix)
    tab = G.table(int(d["table_seeds"][k]), float(d["table_scale"]))
    return O.Expert(w, tab, O.level_resolutions(16, 16, 4096), sc["mins"][k], d[f"w:submodules.{k}.aabb_extent"])


def _sigma_close(a, b):
    a = np.asarray(a); b = np.asarray(b)
    err = np.abs(a - b) / np.maximum(1.0, np.abs(b))
    return float(np.nanmax(err)) if err.size else 0.0


# ---------------------------------------------------------------------------------------------
@pytest.mark.parametrize("name", ["lin_L16_T20", "near_L16_T12", "smooth_L16_T12", "lin_L4_T19",
                                  "lin_L8_T14_r2_512"])
def test_hashgrid_fwd_bit_exact_vs_reference(name):
    ops = _ops()
    d = G.load("hashgrid")
    L, mn, mx, log2T, seed, interp = [int(v) for v in d[f"{name}:cfg"]]
    from adaptive_city_nerf_amd.synthetic import formula_table
    tab = _t(formula_table(L, log2T, 2, seed=seed, scale=0.5))
    y = ops.hashgrid_fwd(_t(d["x01"]), tab, d[f"{name}:resolutions"].tolist(), log2T, 2, interp)
    np.testing.assert_array_equal(y.cpu().numpy(), d[f"{name}:y"])


@pytest.mark.parametrize("name", ["lin_L16_T20", "smooth_L16_T12", "lin_L4_T19"])
@pytest.mark.parametrize("M", [1, 63, 65, 1000, 4095])
def test_hashgrid_fwd_ragged_prefixes_bit_exact(name, M):
    """Point counts off the level-major kernel's 64-point blocks (hashgrid_fwd_f2_lm) and fewer than 16 levels:
    every prefix of the fixture batch gives the fixture's rows bit for bit."""
    ops = _ops()
    d = G.load("hashgrid")
    L, mn, mx, log2T, seed, interp = [int(v) for v in d[f"{name}:cfg"]]
    from adaptive_city_nerf_amd.synthetic import formula_table
    tab = _t(formula_table(L, log2T, 2, seed=seed, scale=0.5))
    y = ops.hashgrid_fwd(_t(d["x01"][:M]), tab, d[f"{name}:resolutions"].tolist(), log2T, 2, interp)
    np.testing.assert_array_equal(y.cpu().numpy(), d[f"{name}:y"][:M])


@pytest.mark.parametrize("interp", [1, 2])
@pytest.mark.parametrize("counts", [(700, 0, 1301), (1, 63, 65), (4096, 5, 2)])
def test_hashgrid_fwd_pairs_bit_exact_vs_single_table(interp, counts):
    """The routed training forward (acn_hashgrid_fwd_pairs: slots grouped by expert, each through its expert's
    table, hashgrid_fwd_pairs_lm) equals acn_hashgrid_fwd of each expert's slice bit for bit, at slot counts off
    the 64-slot blocks and with an empty expert."""
    import ctypes as C
    from adaptive_city_nerf_amd import _lib
    from adaptive_city_nerf_amd._lib import check, ptr
    from adaptive_city_nerf_amd.synthetic import formula_table
    ops = _ops()
    L, log2T = 16, 14
    res = O.level_resolutions(L, 16, 2048).tolist()
    K = len(counts)
    g = torch.Generator().manual_seed(7)
    tabs = [_t(formula_table(L, log2T, 2, seed=11 + k, scale=0.5)) for k in range(K)]
    M = sum(counts)
    x01 = torch.rand(M, 3, generator=g).to(DEV)
    pk = torch.cat([torch.full((c,), k, dtype=torch.int32) for k, c in enumerate(counts)]).to(DEV)
    seg = torch.tensor(np.concatenate([[0], np.cumsum(counts)]), dtype=torch.int64).to(DEV)
    out = torch.full((M, 2 * L), float("nan"), device=DEV)
    tp = (C.c_void_p * K)(*[t.data_ptr() for t in tabs])
    rp = (C.c_int32 * L)(*res)
    check(_lib.lib().acn_hashgrid_fwd_pairs(ptr(x01), ptr(pk), ptr(seg), K, tp, rp, L, log2T, interp, ptr(out),
                                            torch.cuda.current_stream().cuda_stream), "acn_hashgrid_fwd_pairs")
    o = 0
    for k, c in enumerate(counts):
        if c:
            ref = ops.hashgrid_fwd(x01[o:o + c], tabs[k], res, log2T, 2, interp)
            assert torch.equal(out[o:o + c], ref), f"expert {k}"
        o += c


@pytest.mark.parametrize("name", ["near_L16_T12", "smooth_L16_T12", "lin_L8_T14_r2_512"])
def test_hashgrid_bwd_vs_reference(name):
    ops = _ops()
    d = G.load("hashgrid")
    L, mn, mx, log2T, seed, interp = [int(v) for v in d[f"{name}:cfg"]]
    g = ops.hashgrid_bwd(_t(d["x01"]), _t(d[f"{name}:gy"]), d[f"{name}:resolutions"].tolist(), log2T, 2, interp)
    ref = d[f"{name}:gtable"]
    np.testing.assert_allclose(g.cpu().numpy(), ref, rtol=0, atol=2e-5 * max(1.0, float(np.abs(ref).max())))


@pytest.mark.parametrize("levels", [1, 2, 3, 4, 5])
def test_sh_bit_exact_vs_reference(levels):
    ops = _ops()
    d = G.load("sh")
    y = ops.sh_fwd(_t(d["d"]), levels)
    np.testing.assert_array_equal(y.cpu().numpy(), d[f"levels{levels}"])


def test_volume_render_vs_reference():
    ops = _ops()
    d = G.load("volume_render")
    rgb, depth, w, acc = ops.volume_render(_t(d["rgb_sigma"]), _t(d["t_vals"]), _t(d["bg"]))
    np.testing.assert_allclose(rgb.cpu().numpy(), d["a:rgb"], rtol=0, atol=1e-6)
    np.testing.assert_allclose(depth.cpu().numpy(), d["a:depth"], rtol=0, atol=1e-6)
    np.testing.assert_allclose(acc.cpu().numpy(), d["a:acc"], rtol=0, atol=1e-6)
    np.testing.assert_allclose(w.cpu().numpy(), d["a:weights"], rtol=0, atol=2e-7)
    rs = d["rgb_sigma"] * np.float32(3) - np.float32(1)
    rgb, depth, w, acc = ops.volume_render(_t(rs), _t(d["t_vals"]), None, raw_rgb=True, raw_sigma=True,
                                           sigma_scale=2.0)
    np.testing.assert_allclose(rgb.cpu().numpy(), d["b:rgb"], rtol=0, atol=1e-6)
    np.testing.assert_allclose(w.cpu().numpy(), d["b:weights"], rtol=0, atol=2e-7)


@pytest.mark.parametrize("tag", ["k1", "k4"])
def test_field_vs_reference(tag):
    ops = _ops()
    d = G.load(f"render_{tag}")
    mask = G.MASK[tag]
    sc = G.scene()["masks"][mask]
    K = len(sc["centroids"])
    specs = [_spec(d, k, mask) for k in range(K)]
    routing = ops.make_routing(torch.tensor(sc["centroids"]), K, True, float(d["bm"]))
    x = _t(d["field:x_d"])
    y0 = ops.field_fwd(x, [specs[0]], ops.make_routing(torch.tensor(sc["centroids"])[:1], 1, True, float(d["bm"])),
                       active_module=0).cpu().numpy()
    ref0 = d["field:y_expert0"]
    assert np.abs(y0[:, :3] - ref0[:, :3]).max() <= RGB_TOL
    assert _sigma_close(y0[:, 3], ref0[:, 3]) <= SIGMA_TOL
    yc = ops.field_fwd(x, specs, routing).cpu().numpy()
    refc = d["field:y_container"]
    assert np.abs(yc[:, :3] - refc[:, :3]).max() <= RGB_TOL
    assert _sigma_close(yc[:, 3], refc[:, 3]) <= SIGMA_TOL


@pytest.mark.parametrize("tag", ["k1", "k4"])
@pytest.mark.parametrize("variant", ["render", "render_a0", "render_fast", "render_hi"])
@pytest.mark.parametrize("tau", [0.0, 1e-5])
def test_render_stratified_vs_reference(tag, variant, tau):
    ops = _ops()
    d = G.load(f"render_{tag}")
    mask = G.MASK[tag]
    sc = G.scene()["masks"][mask]
    K = len(sc["centroids"])
    prefix = "hiw:" if variant == "render_hi" else "w:"
    if variant == "render_fast":
        specs = [_spec(d, k, mask, weights=G.fast_weights(d, k)) for k in range(K)]
    else:
        specs = [_spec(d, k, mask, prefix=prefix) for k in range(K)]
    active = 0 if variant == "render_a0" else None
    if active is not None:
        specs = [specs[active]]
    routing = ops.make_routing(torch.tensor(sc["centroids"]), K, True, float(d["bm"]))
    bgw = {k[len("bg_mlp."):]: _t(v) for k, v in G.bg_weights(d, prefix).items()}
    bg, keep = ops.make_background("mlp", mlp=bgw)
    rgb, depth, w, acc = ops.render_stratified(_t(d["render:rays"]), 64, specs, routing, active, bg, tau=tau)
    rgb = rgb.cpu().numpy(); depth = depth.cpu().numpy(); w = w.cpu().numpy(); acc = acc.cpu().numpy()
    assert np.abs(rgb - d[f"{variant}:rgb"]).max() <= RGB_TOL
    assert np.abs(depth - d[f"{variant}:depth"]).max() <= 1e-4
    assert np.abs(acc - d[f"{variant}:acc"]).max() <= 1e-4
    assert np.abs(w - d[f"{variant}:weights"]).max() <= 1e-5


def test_get_rays_vs_reference():
    ops = _ops()
    d = G.load("rays")
    sc = G.scene()
    cam = sc["val_cam0"]
    m = sc["masks"]["g22_grid_bm110_ss11"]
    psf = sc["pose_scale_factor"]
    for tag in ("ds16", "ds4"):
        H, W, fx, fy, cx, cy = d[f"{tag}:cam"]
        rays, valid = ops.get_rays_image(int(H), int(W), fx, fy, cx, cy, torch.tensor(cam["c2w"]),
                                         torch.tensor(m["aabb_global"]), DEV,
                                         near_far_override=(0.0 / psf, 100000 / psf))
        rays = rays.cpu().numpy(); valid = valid.cpu().numpy()
        if tag == "ds4":
            rays = rays[d["ds4:sel"]]; valid = valid[d["ds4:sel"]]
        ref = d[f"{tag}:rays"]
        assert np.array_equal(valid, d[f"{tag}:valid"])
        np.testing.assert_array_equal(rays[:, :3], ref[:, :3])
        np.testing.assert_allclose(rays[:, 3:6], ref[:, 3:6], rtol=0, atol=1.2e-7)
        np.testing.assert_allclose(rays[:, 6:], ref[:, 6:], rtol=2e-6, atol=1e-7)


def test_render_full_size_vs_oracle():
    """BASELINE config C2 size (4096 rays x 256 samples, 1 expert): a sampled subset of rays is
    checked against the oracle, and size-independent invariants on all rays."""
    ops = _ops()
    d = G.load("render_k1")
    mask = G.MASK["k1"]
    sc = G.scene()["masks"][mask]
    cam = G.scene()["val_cam0"]
    psf = G.scene()["pose_scale_factor"]
    ds = 0.25
    H = int(round(cam["H"] * ds)); W = int(round(cam["W"] * ds))
    intr = np.array(cam["intrinsics"], np.float32) * np.float32(ds)
    rays_all, valid = O.get_rays(H, W, *intr.tolist(), cam["c2w"], aabb=np.array(sc["aabb_global"], np.float32),
                                 near_far_override=(0.0, 100000 / psf))
    rng = np.random.default_rng(0)
    idx = rng.choice(np.nonzero(valid)[0], 4096, replace=False)
    rays = rays_all[idx]
    specs = [_spec(d, 0, mask, prefix="hiw:")]
    routing = ops.make_routing(torch.tensor(sc["centroids"]), 1, True, float(d["bm"]))
    bgw = {k[len("bg_mlp."):]: _t(v) for k, v in G.bg_weights(d, "hiw:").items()}
    bg, keep = ops.make_background("mlp", mlp=bgw)
    rgb, depth, w, acc = [t.cpu().numpy() for t in ops.render_stratified(_t(rays), 256, specs, routing, None, bg)]
    assert np.all(np.isfinite(rgb)) and np.all((acc >= 0) & (acc <= 1 + 1e-6))
    np.testing.assert_allclose(w.sum(1), acc, rtol=0, atol=2e-6)
    sub = np.arange(0, 4096, 64)
    e = _oracle_expert(d, 0, mask, prefix="hiw:")
    orgb, odepth, ow, oacc = O.render_stratified(rays[sub], 256, [e], np.array(sc["centroids"], np.float32),
                                                 bm=float(d["bm"]), bg_mlp=G.bg_weights(d, "hiw:"))
    assert np.abs(rgb[sub] - orgb).max() <= RGB_TOL
    assert np.abs(acc[sub] - oacc).max() <= 1e-4
    assert np.abs(w[sub] - ow).max() <= 1e-5


def test_invalid_rays_give_nan_like_reference():
    """clamp_rays_near_far marks misses with near=far=+inf; the reference then renders NaN
    (SURVEY §8(a3)).  The fused kernel reproduces it rather than masking."""
    ops = _ops()
    d = G.load("render_k1")
    mask = G.MASK["k1"]
    sc = G.scene()["masks"][mask]
    rays = d["render:rays"][:64].copy()
    rays[::2, 6:] = np.inf
    specs = [_spec(d, 0, mask)]
    routing = ops.make_routing(torch.tensor(sc["centroids"]), 1, True, float(d["bm"]))
    bgw = {k[len("bg_mlp."):]: _t(v) for k, v in G.bg_weights(d).items()}
    bg, keep = ops.make_background("mlp", mlp=bgw)
    rgb, depth, w, acc = ops.render_stratified(_t(rays), 64, specs, routing, None, bg)
    rgb = rgb.cpu().numpy()
    assert np.all(np.isnan(rgb[::2])) and np.all(np.isfinite(rgb[1::2]))


@pytest.mark.parametrize("n", [1, 17, 777, 4096, 8192, 8193])
@pytest.mark.parametrize("jitter", [False, True])
def test_render_ray_order_bit_identical(n, jitter):
    """acn_render_stratified_fwd_ordered sorts small batches by direction (Z-order) and walks them
    in XCD bands; every output must equal the given-order render bit for bit -- including NaN
    rays (inf near/far), a zero and a NaN direction -- on both sides of the re-ordered size cap."""
    ops = _ops()
    d = G.load("render_k1")
    mask = G.MASK["k1"]
    sc = G.scene()["masks"][mask]
    base = d["render:rays"]
    rng = np.random.default_rng(n)
    rays = base[rng.integers(0, base.shape[0], n)].copy()
    if n > 4:
        rays[1, 6:] = np.inf
        rays[2, 3:6] = 0.0
        rays[3, 3:6] = np.nan
    specs = [_spec(d, 0, mask, prefix="hiw:")]
    routing = ops.make_routing(torch.tensor(sc["centroids"]), 1, True, float(d["bm"]))
    bgw = {k[len("bg_mlp."):]: _t(v) for k, v in G.bg_weights(d, "hiw:").items()}
    bg, keep = ops.make_background("mlp", mlp=bgw)
    S = 64
    jit = _t(rng.random((n, S), dtype=np.float32)) if jitter else None
    a = ops.render_stratified(_t(rays), S, specs, routing, None, bg, jitter=jit, reorder=True)
    b = ops.render_stratified(_t(rays), S, specs, routing, None, bg, jitter=jit, reorder=False)
    for x, y in zip(a, b):
        assert np.array_equal(x.cpu().numpy(), y.cpu().numpy(), equal_nan=True)
    # the scratch covers the ray order (n <= 8192) and, for routed K > 2 batches, the split render's ray lists
    assert _ops()._lib.lib().acn_render_order_bytes(n) >= (4 * n if n <= 8192 else 0)
