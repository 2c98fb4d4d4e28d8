"""BASELINE C4 / C5 expert count: the K=8 container (g42 layout) against the
reference's own render_rays / render_image / MetaContainer.forward (tests/golden/render_k8.npz,
make_golden.py gen_k8): every routed render variant, the reference's default table scale
(U(-1e-3, 1e-3), encodings.py:264-268) through the fp16x3 MLP, and the full C4 frame (800x800 x 256
samples, 8 experts) against the C oracle on sampled rays plus size-independent properties.
Tolerances (north star): RGB 1e-4, sigma 1e-5 relative to max(1, |sigma|), weights 1e-5."""
from collections import OrderedDict

import numpy as np
import pytest
import torch

import goldens as G
from oracle import oracle as O

TAG, MASK = "k8", G.MASK["k8"]
DEFAULT_SCALE = 1e-3
VARIANTS = ["render", "render_fast", "render_hi", "render_default"]


def _scale(variant):
    return DEFAULT_SCALE if variant == "render_default" else None


def _expert(d, k, prefix="w:", weights=None, scale=None):
    sc = G.scene()["masks"][MASK]
    w = weights if weights is not None else G.expert_weights(d, k, prefix)
    tab = G.table(int(d["table_seeds"][k]), float(d["table_scale"]) if scale is None else scale)
    return O.Expert(w, tab, O.level_resolutions(16, 16, 4096), sc["mins"][k], d[f"w:submodules.{k}.aabb_extent"])


def _oracle_experts(d, variant):
    K = len(G.scene()["masks"][MASK]["centroids"])
    if variant == "render_fast":
        return [_expert(d, k, weights=G.fast_weights(d, k)) for k in range(K)]
    return [_expert(d, k, "hiw:" if variant == "render_hi" else "w:", scale=_scale(variant)) for k in range(K)]


# ------------------------------------------------------------------------------------------ CPU
def test_fixture_blends_experts():
    """The fixture exercises soft routing: samples blending two experts exist."""
    d = G.load("render_k8")
    h = d["render:experts_per_sample_hist"]
    assert h[1] > 0 and h[2] > 0


@pytest.mark.parametrize("which", ["field", "field_default"])
def test_oracle_field_k8(which):
    d = G.load("render_k8")
    sc = G.scene()["masks"][MASK]
    experts = [_expert(d, k, scale=DEFAULT_SCALE if which == "field_default" else None) for k in range(8)]
    yc = O.container_fwd(experts, np.array(sc["centroids"], np.float32), d["field:x_d"], bm=float(d["bm"]))
    ref = d[f"{which}:y_container"]
    np.testing.assert_allclose(yc[:, :3], ref[:, :3], rtol=0, atol=1e-6)
    np.testing.assert_allclose(yc[:, 3], ref[:, 3], rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("variant", VARIANTS)
def test_oracle_render_k8(variant):
    d = G.load("render_k8")
    sc = G.scene()["masks"][MASK]
    bgw = G.bg_weights(d, "hiw:" if variant == "render_hi" else "w:")
    rgb, depth, w, acc = O.render_stratified(d["render:rays"], 64, _oracle_experts(d, variant),
                                             np.array(sc["centroids"], np.float32), bm=float(d["bm"]), bg_mlp=bgw)
    np.testing.assert_allclose(rgb, d[f"{variant}:rgb"], rtol=0, atol=1e-5)
    np.testing.assert_allclose(depth, d[f"{variant}:depth"], rtol=0, atol=1e-5)
    np.testing.assert_allclose(acc, d[f"{variant}:acc"], rtol=0, atol=1e-5)
    np.testing.assert_allclose(w, d[f"{variant}:weights"], rtol=0, atol=1e-6)


# ------------------------------------------------------------------------------------------ GPU
def _model(d, prefix="w:", scale=None):
    from test_module_api import build_model
    m, gbox = build_model(TAG)
    sd = {k[len(prefix):]: torch.from_numpy(v.copy()) for k, v in d.items() if k.startswith(prefix)}
    for k in range(len(m.submodules)):
        sd[f"submodules.{k}.xyz_encoder.hash_table"] = torch.from_numpy(
            G.table(int(d["table_seeds"][k]), float(d["table_scale"]) if scale is None else scale).copy())
    m.load_state_dict(sd)
    return m.cuda().eval(), gbox


@pytest.mark.gpu
@pytest.mark.parametrize("variant", VARIANTS)
@pytest.mark.parametrize("tau", [0.0, 1e-5])
def test_render_rays_k8_vs_reference(variant, tau):
    """render_rays through the module API: the 8-expert routed fused render (render_slots_kernel)."""
    from adaptive_city_nerf_amd import render_rays
    d = G.load("render_k8")
    m, _ = _model(d, "hiw:" if variant == "render_hi" else "w:", _scale(variant))
    params = None
    if variant == "render_fast":
        params = OrderedDict((k[len("fast:"):], torch.from_numpy(v).cuda()) for k, v in d.items()
                             if k.startswith("fast:"))
    rays = torch.from_numpy(d["render:rays"]).cuda()
    with torch.no_grad():
        rgb, depth, w, acc = render_rays(m, rays, ray_samples=64, params=params, bg_color_default="white",
                                         early_stop_tau=tau)
    assert np.abs(rgb.cpu().numpy() - d[f"{variant}:rgb"]).max() <= 1e-4
    assert np.abs(acc.cpu().numpy() - d[f"{variant}:acc"]).max() <= 1e-4
    assert np.abs(depth.cpu().numpy() - d[f"{variant}:depth"]).max() <= 1e-4
    assert np.abs(w.cpu().numpy() - d[f"{variant}:weights"]).max() <= 1e-5


@pytest.mark.gpu
@pytest.mark.parametrize("variant", ["render", "render_hi"])
@pytest.mark.parametrize("S", [64, 96, 200])
def test_depth_tiled_routed_render_equals_ray_tiles(variant, S):
    """render_wss_kernel (tau = 0: depth tiles -- 16-ray rounds in 16 x 2 tiles up to S = 128, 8-ray rounds in 8 x 4
    tiles above -- unfolded SH-first colour layer, LDS compositing)
    renders every ray bit for bit like render_slots_kernel (taken with an early-termination threshold so small that
    only an underflowed transmittance, whose later samples add exact zeros, can stop a ray): rgb, depth, weights, acc."""
    from adaptive_city_nerf_amd import render_rays
    d = G.load("render_k8")
    m, _ = _model(d, "hiw:" if variant == "render_hi" else "w:")
    rays = torch.from_numpy(d["render:rays"]).cuda()
    with torch.no_grad():
        a = render_rays(m, rays, ray_samples=S, bg_color_default="white")
        b = render_rays(m, rays, ray_samples=S, bg_color_default="white", early_stop_tau=1e-37)
    for x, y, name in zip(a, b, ("rgb", "depth", "weights", "acc")):
        assert torch.equal(x, y), name


def _single_expert_rays(rays, S, sc, bm):
    """Per ray: the one expert every sample routes to with weight exactly 1.0f (else -1), from the
    oracle's routing at the eval t-values (linspace as torch CPU, ray_rendering.py:278-287)."""
    i = np.arange(S)
    step = np.float32(1.0) / np.float32(S - 1)
    u = np.where(i < S // 2, (step * i.astype(np.float32)).astype(np.float32),
                 (np.float32(1.0) - step * (S - 1 - i).astype(np.float32)).astype(np.float32)).astype(np.float32)
    near, far = rays[:, 6:7], rays[:, 7:8]
    t = (near * (np.float32(1) - u) + far * u).astype(np.float32)
    pts = (rays[:, None, :3] + rays[:, None, 3:6] * t[..., None]).astype(np.float32)
    W, _ = O.routing(pts.reshape(-1, 3), np.array(sc["centroids"], np.float32), sc["cluster_2d"], bm)
    W = W.reshape(rays.shape[0], S, -1)
    one = ((W > 0).sum(-1) == 1) & ((W == 1.0) | (W == 0.0)).all(-1)
    k = W.argmax(-1)
    ok = one.all(1) & (k == k[:, :1]).all(1)
    return np.where(ok, k[:, 0], -1)


@pytest.mark.gpu
def test_single_expert_rays_bit_identical_to_active_module():
    """render_slots_kernel's single-expert fast path (every sample of the ray routed to one expert
    with weight exactly 1.0: the blend 0 + y_k * 1.0f is y_k) renders those rays bit for bit like the
    active_module render of that expert (render_kernel, same field tile and compositing code)."""
    from adaptive_city_nerf_amd import render_rays
    d = G.load("render_k8")
    m, _ = _model(d)
    sc = G.scene()["masks"][MASK]
    rays = d["render:rays"]
    ks = _single_expert_rays(rays, 64, sc, float(d["bm"]))
    vals, cnt = np.unique(ks[ks >= 0], return_counts=True)
    assert cnt.sum() >= rays.shape[0] // 2, "fixture rays should be mostly single-expert"
    k = int(vals[np.argmax(cnt)])
    sel = torch.from_numpy(rays[ks == k]).cuda()
    with torch.no_grad():
        a = render_rays(m, sel, ray_samples=64, bg_color_default="white")
        b = render_rays(m, sel, ray_samples=64, bg_color_default="white", active_module=k)
    for x, y in zip(a, b):
        assert torch.equal(x, y)


@pytest.mark.gpu
@pytest.mark.parametrize("which", ["field", "field_default"])
def test_container_forward_k8_vs_reference(which):
    d = G.load("render_k8")
    m, _ = _model(d, scale=DEFAULT_SCALE if which == "field_default" else None)
    x = torch.from_numpy(d["field:x_d"]).cuda()
    with torch.no_grad():
        y = m(x).cpu().numpy()
    ref = d[f"{which}:y_container"]
    assert np.abs(y[:, :3] - ref[:, :3]).max() <= 1e-4
    assert (np.abs(y[:, 3] - ref[:, 3]) / np.maximum(1, np.abs(ref[:, 3]))).max() <= 1e-5


@pytest.mark.gpu
def test_render_image_k8_vs_reference():
    from adaptive_city_nerf_amd import render_image
    d = G.load("render_k8")
    m, gbox = _model(d, "hiw:")
    cam = G.scene()["val_cam0"]
    ds = 1.0 / 32
    H, W = [int(v) for v in d["image:hw"]]
    intr = torch.tensor(cam["intrinsics"], dtype=torch.float32) * ds
    img, depth, acc = render_image(m, H=H, W=W, fx=float(intr[0]), fy=float(intr[1]), cx=float(intr[2]),
                                   cy=float(intr[3]), c2w=torch.tensor(cam["c2w"]), scene_box=gbox, ray_samples=32,
                                   chunk_points=1 << 16)
    assert np.abs(img.cpu().numpy() - d["image:rgb"]).max() <= 1e-4
    assert np.abs(acc.cpu().numpy() - d["image:acc"]).max() <= 1e-4
    assert np.nanmax(np.abs(depth.cpu().numpy() - d["image:depth"])) <= 1e-4


@pytest.mark.gpu
@pytest.mark.parametrize("S", [256, 96])
def test_c4_full_frame_vs_oracle(S):
    """BASELINE C4 at full size: one 800x800 frame x S samples through the 8-expert container
    (render_image, the bench's workload).  400 sampled pixels against the C oracle; on all 640,000
    rays: finite, acc in [0, 1], rgb in [0, 1]; the frame equals the concatenation of renders of its
    halves (ray independence)."""
    from adaptive_city_nerf_amd import render_image, render_rays
    from adaptive_city_nerf_amd import ops
    d = G.load("render_k8")
    m, gbox = _model(d, "hiw:")
    cam = G.scene()["val_cam0"]
    H = W = 800
    s = min(H / cam["H"], W / cam["W"])
    intr = [float(cam["intrinsics"][0] * s), float(cam["intrinsics"][1] * s), W / 2.0, H / 2.0]
    c2w = torch.tensor(cam["c2w"])
    img, depth, acc = render_image(m, H=H, W=W, fx=intr[0], fy=intr[1], cx=intr[2], cy=intr[3], c2w=c2w,
                                   scene_box=gbox, ray_samples=S)
    img = img.cpu().numpy().reshape(-1, 3); acc = acc.cpu().numpy()
    rays, valid = ops.get_rays_image(H, W, *intr, c2w, gbox.aabb, "cuda", near_far_override=(None, None))
    v = valid.cpu().numpy()
    assert v.mean() > 0.5
    assert np.all(np.isfinite(img[v])) and np.all((img[v] >= 0) & (img[v] <= 1))
    assert np.all((acc[v] >= 0) & (acc[v] <= 1 + 1e-6))
    # ray independence: the two halves rendered separately give the same rows bit for bit
    r = rays
    with torch.no_grad():
        h0 = render_rays(m, r[: r.shape[0] // 2].contiguous(), ray_samples=S, _want_weights=False)[0]
    np.testing.assert_array_equal(np.clip(h0.cpu().numpy(), 0, 1)[v[: r.shape[0] // 2]],
                                  img[: r.shape[0] // 2][v[: r.shape[0] // 2]])
    rng = np.random.default_rng(S)
    idx = rng.choice(np.nonzero(v)[0], 400, replace=False)
    sc = G.scene()["masks"][MASK]
    orgb, odepth, ow, oacc = O.render_stratified(rays.cpu().numpy()[idx], S, _oracle_experts(d, "render_hi"),
                                                 np.array(sc["centroids"], np.float32), bm=float(d["bm"]),
                                                 bg_mlp=G.bg_weights(d, "hiw:"), want_weights=False)
    assert np.abs(img[idx] - np.clip(orgb, 0, 1)).max() <= 1e-4
    assert np.abs(acc[idx] - oacc).max() <= 1e-4
