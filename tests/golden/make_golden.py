#!/usr/bin/env python3
"""Generate the committed golden fixtures by running the REFERENCE's own code (this container only).

Run:  python tests/golden/make_golden.py   (needs /root/reference; never runs on the GPU box)

The reference is imported from /root/reference with the stubs of _refstubs.py;
its pure-Torch CPU path (tinycudann absent) is the parity oracle.  Only inputs and outputs are
written (npz, loadable with allow_pickle=False) plus scene geometry as JSON; no reference source
is copied.  Hash tables are formula-filled (adaptive_city_nerf_amd/synthetic.py) so the 128 MiB
tables are regenerated from (seed, scale) instead of stored.
"""
from __future__ import annotations

import json
import os
import sys
from pathlib import Path

import numpy as np
import torch

HERE = Path(__file__).resolve().parent
REPO = HERE.parent.parent
REF = Path(os.environ.get("ACN_REFERENCE", "/root/reference"))
sys.path.insert(0, str(REPO))
sys.path.insert(0, str(HERE))

import _refstubs  # noqa: E402

_refstubs.install()
sys.path.insert(0, str(REF))

import warnings  # noqa: E402

warnings.filterwarnings("ignore")

from adaptive_city_nerf_amd.synthetic import formula_table  # noqa: E402
from models.encodings import HashGridEncoder, SHEncoder  # noqa: E402
from models.inr.meta_container import MetaContainer  # noqa: E402
from nerfs.ray_rendering import render_rays, volume_render, render_image  # noqa: E402
from nerfs.ray_sampling import clamp_rays_near_far, get_ray_directions, get_rays  # noqa: E402
from nerfs.scene_box import SceneBox  # noqa: E402

DATA = REF / "data" / "drz" / "out" / "example"
TABLE_SCALE = 0.5          # U(-0.5, 0.5) so sigma/colour vary
BM_RUNTIME = 1.05          # nerf_runner.py:150  min(max(1, --bm=1.05), params 1.1)
F32 = np.float32


def _np(t: torch.Tensor) -> np.ndarray:
    return t.detach().cpu().numpy().copy()


def save(name: str, **arrays) -> None:
    meta = {"torch": torch.__version__, "numpy": np.__version__, "generator": "tests/golden/make_golden.py"}
    arrays["_meta"] = np.array(json.dumps(meta))
    np.savez_compressed(HERE / f"{name}.npz", **arrays)
    print("wrote", name, len(arrays), "arrays")


# ----------------------------------------------------------------------------------------------
def scene_json() -> dict:
    coords = torch.load(DATA / "coordinates.pt", map_location="cpu", weights_only=True)
    vmeta = torch.load(DATA / "val" / "metadata" / "000000.pt", map_location="cpu", weights_only=True)
    out = {
        "pose_scale_factor": float(coords["pose_scale_factor"]),
        "val_cam0": {
            "H": int(vmeta["H"]), "W": int(vmeta["W"]),
            "c2w": _np(vmeta["c2w"].float()).tolist(),
            "intrinsics": _np(vmeta["intrinsics"].float()).tolist(),
        },
        "masks": {},
    }
    for mask in ["g11_grid_bm110_ss11", "g22_grid_bm110_ss11"]:
        p = torch.load(DATA / "masks" / mask / "params.pt", map_location="cpu", weights_only=True)
        b = torch.load(DATA / "masks" / mask / "scene_boxes.pt", map_location="cpu", weights_only=True)
        out["masks"][mask] = {
            "centroids": _np(p["centroids"].float()).tolist(),
            "cluster_2d": bool(p["cluster_2d"]),
            "boundary_margin": float(p["boundary_margin"]),
            "aabb_global": _np(b["aabb_global"].float()).tolist(),
            "mins": _np(b["mins"].float()).tolist(),
            "maxs": _np(b["maxs"].float()).tolist(),
        }
    # BASELINE C4's 4x2 layout: the reference ships no g42 mask set; centroids by the
    # _grid_centroids rule (equal to the reference's own _grid_centroids output, clusters.npz
    # cent_grid42_2d), boxes by synthetic.grid_layout's Voronoi-cell rule
    from adaptive_city_nerf_amd.synthetic import grid_layout
    out["masks"]["g42_synthetic"] = grid_layout(4, 2, out)
    return out


def build_container(scene: dict, mask: str, seed: int = 0, table_seed0: int = 100, occ_conf=None):
    m = scene["masks"][mask]
    K = len(m["centroids"])
    gbox = SceneBox(aabb=torch.tensor(m["aabb_global"], dtype=torch.float32))
    boxes = [SceneBox(aabb=torch.tensor([m["mins"][k], m["maxs"][k]], dtype=torch.float32)) for k in range(K)]
    hash_conf = {"levels": 16, "features_per_level": 2, "log2_hashmap_size": 20,
                 "max_res": 4096, "min_res": 16, "interpolation": "Linear"}
    torch.manual_seed(seed)
    model = MetaContainer(
        num_submodules=K, centroids=torch.tensor(m["centroids"], dtype=torch.float32),
        aabb=gbox.aabb, nerf_variant="instant", boundary_margin=min(max(1.0, BM_RUNTIME), m["boundary_margin"]),
        cluster_2d=m["cluster_2d"], joint_training=False, use_bg_nerf=True, bg_hidden=32,
        bg_encoding="spherical", occ_conf=occ_conf or {"use_occ": False}, expert_box_list=boxes, hidden=64,
        sigma_depth=2, color_depth=2, dir_encoding="spherical", color_hidden=64,
        use_sigmoid_rgb=True, hash_enc_conf=hash_conf,
    )
    with torch.no_grad():
        for k, sub in enumerate(model.submodules):
            tab = formula_table(16, 20, 2, seed=table_seed0 + k, scale=TABLE_SCALE)
            sub.xyz_encoder.hash_table.data.copy_(torch.from_numpy(tab))
    model.eval()
    return model, gbox


def weights_dict(model) -> dict:
    """MLP + background weights keyed by the reference state-dict names (tables excluded)."""
    out = {}
    for k, v in model.state_dict().items():
        if k.endswith("hash_table"):
            continue
        out["w:" + k] = _np(v.float()).copy()   # copy: state_dict tensors alias live params
    return out


def val_rays(scene: dict, mask: str, downscale: float) -> torch.Tensor:
    cam = scene["val_cam0"]
    H = int(round(cam["H"] * downscale)); W = int(round(cam["W"] * downscale))
    fx, fy, cx, cy = (torch.tensor(cam["intrinsics"]) * downscale).tolist()
    intr = torch.tensor(cam["intrinsics"], dtype=torch.float32) * downscale
    fx, fy, cx, cy = [float(v) for v in intr]
    dirs = get_ray_directions(H, W, fx, fy, cx, cy, True, device=torch.device("cpu"))
    m = scene["masks"][mask]
    gbox = SceneBox(aabb=torch.tensor(m["aabb_global"], dtype=torch.float32))
    rays = get_rays(dirs, torch.tensor(cam["c2w"], dtype=torch.float32), scene_box=gbox).view(-1, 8)
    psf = scene["pose_scale_factor"]
    rays, valid = clamp_rays_near_far(rays, near_far_override=(0.0 / psf, 100000 / psf))
    return rays, valid, (H, W, fx, fy, cx, cy)


# ----------------------------------------------------------------------------------------------
def gen_hashgrid() -> None:
    g = torch.Generator().manual_seed(0)
    x = torch.rand(4096, 3, generator=g)
    edge = torch.tensor([[0.0, 0.0, 0.0], [1.0, 1.0, 1.0], [1e-6, 1e-6, 1e-6], [1 - 1e-6, 0.5, 1e-6],
                         [0.5, 0.5, 0.5], [0.25, 0.75, 0.125], [1.0 / 16, 2.0 / 23, 3.0 / 33],
                         [4095.0 / 4095, 7.0 / 4095, 0.999999]], dtype=torch.float32)
    x = torch.cat([x, edge], 0)
    variants = [
        ("lin_L16_T20", dict(levels=16, min_res=16, max_res=4096, log2_hashmap_size=20, interpolation="Linear"), 7),
        ("near_L16_T12", dict(levels=16, min_res=16, max_res=4096, log2_hashmap_size=12, interpolation="Nearest"), 8),
        ("smooth_L16_T12", dict(levels=16, min_res=16, max_res=4096, log2_hashmap_size=12, interpolation="Smoothstep"), 9),
        ("lin_L4_T19", dict(levels=4, min_res=16, max_res=4096, log2_hashmap_size=19, interpolation="Linear"), 10),
        ("lin_L8_T14_r2_512", dict(levels=8, min_res=2, max_res=512, log2_hashmap_size=14, interpolation="Linear"), 11),
    ]
    out = {"x01": _np(x)}
    for name, kw, seed in variants:
        enc = HashGridEncoder(features_per_level=2, implementation="torch", **kw)
        tab = formula_table(kw["levels"], kw["log2_hashmap_size"], 2, seed=seed, scale=TABLE_SCALE)
        with torch.no_grad():
            enc.hash_table.data.copy_(torch.from_numpy(tab))
            y = enc(x)
        out[f"{name}:y"] = _np(y)
        out[f"{name}:resolutions"] = _np(enc.level_resolutions)
        out[f"{name}:cfg"] = np.array([kw["levels"], kw["min_res"], kw["max_res"], kw["log2_hashmap_size"], seed,
                                       {"Nearest": 0, "Linear": 1, "Smoothstep": 2}[kw["interpolation"]]], np.int64)
        # backward: d/dtable of <y, g> for a fixed cotangent (scatter-add semantics of index backward)
        if kw["log2_hashmap_size"] <= 14:
            enc.hash_table.grad = None
            gy = torch.randn(y.shape, generator=g)
            y2 = enc(x)
            (y2 * gy).sum().backward()
            out[f"{name}:gy"] = _np(gy)
            out[f"{name}:gtable"] = _np(enc.hash_table.grad)
    save("hashgrid", **out)


def gen_sh() -> None:
    g = torch.Generator().manual_seed(1)
    d = torch.randn(1024, 3, generator=g) * 3.0
    d[0] = torch.tensor([0.0, 0.0, 0.0]); d[1] = torch.tensor([0.0, 0.0, -1.0]); d[2] = torch.tensor([1e-12, 0, 0])
    out = {"d": _np(d)}
    for lv in range(1, 6):
        enc = SHEncoder(levels=lv, implementation="torch")
        out[f"levels{lv}"] = _np(enc(d))
    save("sh", **out)


def gen_volume_render() -> None:
    g = torch.Generator().manual_seed(2)
    N, S = 256, 64
    rgb = torch.rand(N, S, 3, generator=g) * 1.4 - 0.2                 # exercises clamp(0,1)
    sig = torch.exp(torch.rand(N, S, generator=g) * 14 - 7) - 0.01     # (-0.01, ~1e3): clamp_min(0)
    sig[:8] *= 1e3                                                      # saturated rays
    rgb_sigma = torch.cat([rgb, sig[..., None]], -1)
    near = torch.rand(N, 1, generator=g) * 0.1
    steps = torch.rand(N, S, generator=g) * 0.01
    steps[:, 5] = 1e-6                                                  # exercises the 1e-4 clamp
    t_vals = near + torch.cumsum(steps, 1)
    bg = torch.rand(N, 3, generator=g)
    a = volume_render(rgb_sigma, t_vals, bg_rgb=bg)
    b = volume_render(rgb_sigma * 3 - 1, t_vals, bg_rgb=None, raw_rgb=True, raw_sigma=True, sigma_scale=2.0)
    out = {"rgb_sigma": _np(rgb_sigma), "t_vals": _np(t_vals), "bg": _np(bg)}
    for tag, res in (("a", a), ("b", b)):
        for nm, v in zip(("rgb", "depth", "weights", "acc"), res):
            out[f"{tag}:{nm}"] = _np(v)
    save("volume_render", **out)


def gen_field_and_render(scene: dict) -> None:
    # --- single expert (g11): field forward on random points + end-to-end render --------------
    for mask, tag in (("g11_grid_bm110_ss11", "k1"), ("g22_grid_bm110_ss11", "k4")):
        model, gbox = build_container(scene, mask)
        K = len(model.submodules)
        w = weights_dict(model)
        g = torch.Generator().manual_seed(3)
        out = dict(w)
        # field samples inside the global box (+ a few outside to exercise the clamp)
        lo = gbox.min; hi = gbox.max
        x = lo + (hi - lo) * (torch.rand(4096, 3, generator=g) * 1.1 - 0.05)
        d = torch.randn(4096, 3, generator=g)
        x_d = torch.cat([x, d], -1)
        with torch.no_grad():
            y_expert0 = model.submodules[0](x_d)
            y_cont = model(x_d)
        out.update({"field:x_d": _np(x_d), "field:y_expert0": _np(y_expert0), "field:y_container": _np(y_cont)})
        # rays from val camera 0 at downscale 0.25, 512 seeded rays, S=64
        rays, valid, cam = val_rays(scene, mask, 0.25)
        rv = rays[valid]
        perm = torch.randperm(rv.shape[0], generator=torch.Generator().manual_seed(0))[:512]
        r512 = rv[perm].contiguous()
        with torch.no_grad():
            res = render_rays(model, r512, ray_samples=64, params=None, active_module=None,
                              bg_color_default="white", chunk=1_000_000)
            res_a0 = render_rays(model, r512, ray_samples=64, params=None, active_module=0,
                                 bg_color_default="white", chunk=1_000_000)
        out["render:rays"] = _np(r512)
        for nm, v in zip(("rgb", "depth", "weights", "acc"), res):
            out[f"render:{nm}"] = _np(v)
        for nm, v in zip(("rgb", "depth", "weights", "acc"), res_a0):
            out[f"render_a0:{nm}"] = _np(v)
        # fast weights: perturbed MLP params passed through `params` (meta_core.py:26-66 style)
        gp = torch.Generator().manual_seed(4)
        fast = {}
        for name, p in model.meta_named_parameters():
            fast[name] = (p.detach() + 0.05 * torch.randn(p.shape, generator=gp)).float()
        with torch.no_grad():
            resf = render_rays(model, r512, ray_samples=64, params=fast, active_module=None,
                               bg_color_default="white", chunk=1_000_000)
        for name, v in fast.items():
            out["fast:" + name] = _np(v)
        for nm, v in zip(("rgb", "depth", "weights", "acc"), resf):
            out[f"render_fast:{nm}"] = _np(v)
        # high-contrast variant: MLP weights scaled x3 in place, so sigma spans orders of magnitude
        # and colours saturate (a far stronger parity check than the near-constant default init)
        with torch.no_grad():
            for name, p in model.meta_named_parameters():
                if name.endswith("weight"):
                    p.mul_(3.0)
            for sub in model.submodules:
                sub.sigma_head.bias.fill_(0.5)
            resh = render_rays(model, r512, ray_samples=64, params=None, active_module=None,
                               bg_color_default="white", chunk=1_000_000)
            y_hi = model(x_d)
        for k2, v2 in weights_dict(model).items():
            out["hi" + k2] = v2
        out["field_hi:y_container"] = _np(y_hi)
        for nm, v in zip(("rgb", "depth", "weights", "acc"), resh):
            out[f"render_hi:{nm}"] = _np(v)
        # full (small) frame through render_image at downscale 1/32 (48x64 rays, S=32)
        cam0 = scene["val_cam0"]; ds = 1.0 / 32
        H = int(round(cam0["H"] * ds)); W = int(round(cam0["W"] * ds))
        intr = torch.tensor(cam0["intrinsics"], dtype=torch.float32) * ds
        with torch.no_grad():
            img, dep, acc = render_image(model, H=H, W=W, fx=float(intr[0]), fy=float(intr[1]), cx=float(intr[2]),
                                         cy=float(intr[3]), c2w=torch.tensor(cam0["c2w"], dtype=torch.float32),
                                         scene_box=gbox, ray_samples=32, chunk_points=1 << 16)
        out.update({"image:rgb": _np(img), "image:depth": _np(dep), "image:acc": _np(acc),
                    "image:hw": np.array([H, W], np.int64)})
        out["table_seeds"] = np.array([100 + k for k in range(K)], np.int64)
        out["table_scale"] = np.array(TABLE_SCALE, np.float64)
        out["bm"] = np.array(model.boundary_margin, np.float64)
        save(f"render_{tag}", **out)
        del model


def gen_k8(scene: dict) -> None:
    """BASELINE C4/C5 expert count: the K=8 container (g42 layout) through the reference's
    render_rays (soft routing, every expert's weights / tables distinct) on 512 rays x 64 samples of
    val camera 0 at downscale 0.25, the x3 high-contrast variant, fast weights, the same rays through
    the reference's DEFAULT table init scale (U(-1e-3, 1e-3), encodings.py:264-268; formula-filled),
    and a small render_image frame.  Also a K=8 field fixture on random points."""
    mask = "g42_synthetic"
    model, gbox = build_container(scene, mask)
    K = len(model.submodules)
    out = dict(weights_dict(model))
    g = torch.Generator().manual_seed(31)
    lo = gbox.min; hi = gbox.max
    x = lo + (hi - lo) * (torch.rand(4096, 3, generator=g) * 1.1 - 0.05)
    d = torch.randn(4096, 3, generator=g)
    x_d = torch.cat([x, d], -1)
    with torch.no_grad():
        out["field:y_container"] = _np(model(x_d))
    out["field:x_d"] = _np(x_d)
    rays, valid, cam = val_rays(scene, mask, 0.25)
    rv = rays[valid]
    perm = torch.randperm(rv.shape[0], generator=torch.Generator().manual_seed(0))[:512]
    r512 = rv[perm].contiguous()
    out["render:rays"] = _np(r512)
    with torch.no_grad():
        res = render_rays(model, r512, ray_samples=64, params=None, active_module=None, bg_color_default="white",
                          chunk=1_000_000)
        # routing statistics of these samples (how many experts each sample blends)
        t = torch.linspace(0, 1, 64)
        pts = (r512[:, None, :3] + r512[:, None, 3:6] * (r512[:, None, 6:7] * (1 - t[None, :, None])
                                                          + r512[:, None, 7:8] * t[None, :, None])).reshape(-1, 3)
        W, _ = model._routing(pts)
        out["render:experts_per_sample_hist"] = _np(torch.bincount((W > 0).sum(1), minlength=K + 1))
    for nm, v in zip(("rgb", "depth", "weights", "acc"), res):
        out[f"render:{nm}"] = _np(v)
    gp = torch.Generator().manual_seed(4)
    fast = {}
    for name, p in model.meta_named_parameters():
        fast[name] = (p.detach() + 0.05 * torch.randn(p.shape, generator=gp)).float()
    with torch.no_grad():
        resf = render_rays(model, r512, ray_samples=64, params=fast, active_module=None, bg_color_default="white",
                           chunk=1_000_000)
    for name, v in fast.items():
        out["fast:" + name] = _np(v)
    for nm, v in zip(("rgb", "depth", "weights", "acc"), resf):
        out[f"render_fast:{nm}"] = _np(v)
    # the reference's default table scale (1e-3): hash features ~1e-3
    with torch.no_grad():
        for k, sub in enumerate(model.submodules):
            sub.xyz_encoder.hash_table.copy_(torch.from_numpy(formula_table(16, 20, 2, seed=100 + k, scale=1e-3)))
        resd = render_rays(model, r512, ray_samples=64, params=None, active_module=None, bg_color_default="white",
                           chunk=1_000_000)
        out["field_default:y_container"] = _np(model(x_d))
    for nm, v in zip(("rgb", "depth", "weights", "acc"), resd):
        out[f"render_default:{nm}"] = _np(v)
    with torch.no_grad():
        for k, sub in enumerate(model.submodules):
            sub.xyz_encoder.hash_table.copy_(torch.from_numpy(formula_table(16, 20, 2, seed=100 + k, scale=TABLE_SCALE)))
        for name, p in model.meta_named_parameters():
            if name.endswith("weight"):
                p.mul_(3.0)
        for sub in model.submodules:
            sub.sigma_head.bias.fill_(0.5)
        resh = render_rays(model, r512, ray_samples=64, params=None, active_module=None, bg_color_default="white",
                           chunk=1_000_000)
    for k2, v2 in weights_dict(model).items():
        out["hi" + k2] = v2
    for nm, v in zip(("rgb", "depth", "weights", "acc"), resh):
        out[f"render_hi:{nm}"] = _np(v)
    cam0 = scene["val_cam0"]; ds = 1.0 / 32
    H = int(round(cam0["H"] * ds)); W = int(round(cam0["W"] * ds))
    intr = torch.tensor(cam0["intrinsics"], dtype=torch.float32) * ds
    with torch.no_grad():
        img, dep, acc = render_image(model, H=H, W=W, fx=float(intr[0]), fy=float(intr[1]), cx=float(intr[2]),
                                     cy=float(intr[3]), c2w=torch.tensor(cam0["c2w"], dtype=torch.float32),
                                     scene_box=gbox, ray_samples=32, chunk_points=1 << 16)
    out.update({"image:rgb": _np(img), "image:depth": _np(dep), "image:acc": _np(acc),
                "image:hw": np.array([H, W], np.int64)})
    out["table_seeds"] = np.array([100 + k for k in range(K)], np.int64)
    out["table_scale"] = np.array(TABLE_SCALE, np.float64)
    out["bm"] = np.array(model.boundary_margin, np.float64)
    save("render_k8", **out)


def gen_train_k8(scene: dict) -> None:
    """BASELINE C5: runtime_adapt updates (runtime_adapt.py:286-309) of the K=8 routed container
    (no active_module: soft routing, every hit expert and the background head train) on batches of
    1000 rays x 96 samples, jitter injected; loss, clip norm, MLP gradients, sampled table-row
    gradients + per-level checksums, parameters after each Adam step (3 steps)."""
    from types import SimpleNamespace
    from common.utils import get_optimizer
    from nerfs.losses import compute_mse_loss
    mask = "g42_synthetic"
    model, gbox = build_container(scene, mask)
    K = len(model.submodules)
    out = dict(weights_dict(model))
    S, NR = 96, 1000
    P = SimpleNamespace(ray_samples=S, chunk_points=4_000_000, color_space="linear", optimizer="adam", lr=1e-4,
                        encoding_lr=0.01, sigma_lr=0.002, color_lr=0.002, bg_lr=0.001, weight_decay=0.0)
    opt = get_optimizer(P, model)
    rays, valid, _ = val_rays(scene, mask, 0.25)
    rv = rays[valid]
    g = torch.Generator().manual_seed(41)
    rows_g = torch.Generator().manual_seed(42)
    sample_rows = torch.randint(0, 16 << 20, (K, 2048), generator=rows_g)
    out["train:rows"] = _np(sample_rows)
    model.train()
    real_rand_like = torch.rand_like
    for step in range(3):
        perm = torch.randperm(rv.shape[0], generator=g)[:NR]
        r = rv[perm].contiguous()
        rgbs = torch.rand(NR, 3, generator=g)
        u = torch.rand(NR, S, generator=g)
        torch.rand_like = lambda t, *a, **k: u.clone() if tuple(t.shape) == tuple(u.shape) else real_rand_like(t, *a, **k)
        try:
            opt.zero_grad()
            loss = compute_mse_loss(P, model=model, data={"rays": r, "rgbs": rgbs}, params=None, active_module=None,
                                    reduction="mean")
            loss.backward()
        finally:
            torch.rand_like = real_rand_like
        pre = f"train{step}:"
        out[pre + "rays"] = _np(r); out[pre + "rgbs"] = _np(rgbs); out[pre + "u"] = _np(u)
        out[pre + "loss"] = np.array(float(loss.detach()), np.float64)
        for name, prm in model.named_parameters():
            if prm.grad is None:
                continue
            if name.endswith("hash_table"):
                k = int(name.split(".")[1])
                gt = prm.grad.detach()
                out[pre + f"grad_rows:{k}"] = _np(gt[sample_rows[k]])
                lv = gt.view(16, -1)
                out[pre + f"grad_level_sum:{k}"] = _np(lv.double().sum(1))
                out[pre + f"grad_level_sumsq:{k}"] = _np((lv.double() ** 2).sum(1))
                out[pre + f"grad_nnz:{k}"] = np.array(int((gt != 0).sum()), np.int64)
            else:
                out[pre + "grad:" + name] = _np(prm.grad)
        total = torch.nn.utils.clip_grad_norm_(model.parameters(), 1.0)
        out[pre + "total_norm"] = np.array(float(total), np.float64)
        opt.step()
        for name, prm in model.named_parameters():
            if name.endswith("hash_table"):
                k = int(name.split(".")[1])
                out[pre + f"table_rows:{k}"] = _np(prm.detach()[sample_rows[k]])
                out[pre + f"table_level_sum:{k}"] = _np(prm.detach().view(16, -1).double().sum(1))
            else:
                out[pre + "param:" + name] = _np(prm)
        print("train_k8 step", step, "loss", float(loss), "norm", float(total),
              "experts with grads", [k for k, s in enumerate(model.submodules) if s.xyz_encoder.hash_table.grad is not None])
    out["table_seeds"] = np.array([100 + k for k in range(K)], np.int64)
    out["table_scale"] = np.array(TABLE_SCALE, np.float64)
    out["bm"] = np.array(model.boundary_margin, np.float64)
    save("train_k8", **out)


def gen_routing(scene: dict) -> None:
    m = scene["masks"]["g22_grid_bm110_ss11"]
    K = len(m["centroids"])
    gbox = SceneBox(aabb=torch.tensor(m["aabb_global"], dtype=torch.float32))
    boxes = [SceneBox(aabb=torch.tensor([m["mins"][k], m["maxs"][k]], dtype=torch.float32)) for k in range(K)]
    g = torch.Generator().manual_seed(5)
    n = 8192
    pts = torch.empty(n, 3)
    pts[:, 0] = torch.rand(n, generator=g) * 0.5
    yz = torch.rand(n, 2, generator=g) * 2.2 - 1.1
    # concentrate half of the points in a thin band around the Voronoi bisectors y=0 / z=0
    band = torch.rand(n // 2, 2, generator=g) * 0.1 - 0.05
    yz[: n // 4, 0] = band[: n // 4, 0]
    yz[n // 4: n // 2, 1] = band[n // 4:, 1]
    pts[:, 1:] = yz
    out = {"pts": _np(pts)}
    for bm in (1.05, 1.0):
        torch.manual_seed(0)
        cont = MetaContainer(
            num_submodules=K, centroids=torch.tensor(m["centroids"]), aabb=gbox.aabb, boundary_margin=bm,
            cluster_2d=True, use_bg_nerf=False, occ_conf={"use_occ": False}, expert_box_list=boxes,
            hidden=8, sigma_depth=1, color_depth=1, color_hidden=8, geo_feat_dim=3,
            hash_enc_conf={"levels": 2, "log2_hashmap_size": 8},
        )
        W, hard = cont._routing(pts)
        if W is not None:
            out[f"bm{bm}:W"] = _np(W)
        else:
            out[f"bm{bm}:hard"] = _np(hard)
    out["centroids"] = np.array(m["centroids"], F32)
    save("routing", **out)


def gen_rays(scene: dict) -> None:
    out = {}
    for ds, tag in ((1.0 / 16, "ds16"), (0.25, "ds4")):
        rays, valid, cam = val_rays(scene, "g22_grid_bm110_ss11", ds)
        H, W, fx, fy, cx, cy = cam
        dirs = get_ray_directions(H, W, fx, fy, cx, cy, True, device=torch.device("cpu"))
        if tag == "ds4":       # keep the fixture small: every 7th ray of the 384x512 frame
            sel = torch.arange(0, rays.shape[0], 7)
            out[f"{tag}:sel"] = _np(sel)
            rays = rays[sel]; valid = valid[sel]; dirs = dirs.view(-1, 3)[sel]
        out[f"{tag}:rays"] = _np(rays)
        out[f"{tag}:valid"] = _np(valid)
        out[f"{tag}:dirs"] = _np(dirs.reshape(-1, 3))
        out[f"{tag}:cam"] = np.array([H, W, fx, fy, cx, cy], np.float64)
    # a synthetic camera whose rays miss the box (invalid -> +inf near/far; NaN downstream, §8(a3))
    m = scene["masks"]["g22_grid_bm110_ss11"]
    gbox = SceneBox(aabb=torch.tensor(m["aabb_global"], dtype=torch.float32))
    c2w = torch.tensor([[1.0, 0, 0, 5.0], [0, 1.0, 0, 5.0], [0, 0, 1.0, 5.0]])
    dirs = get_ray_directions(8, 8, 4.0, 4.0, 4.0, 4.0, False, device=torch.device("cpu"))
    r = get_rays(dirs, c2w, scene_box=gbox).view(-1, 8)
    r2, v2 = clamp_rays_near_far(r, near_far_override=(None, None))
    out.update({"miss:rays_raw": _np(r), "miss:rays": _np(r2), "miss:valid": _np(v2)})
    save("rays", **out)


def gen_train(scene: dict) -> None:
    """SURVEY §8(c) fixture (7): runtime_adapt steps (runtime_adapt.py:288-313) of the K=4
    container on 256 rays x 32 samples, with the training-mode jitter injected (the reference draws
    it with torch.rand_like, ray_rendering.py:286): loss, clip norm, gradients (MLP tensors whole,
    hash-table rows sampled + per-level checksums) and parameters after each Adam step."""
    from types import SimpleNamespace
    from common.utils import get_optimizer
    from nerfs.losses import compute_mse_loss
    mask = "g22_grid_bm110_ss11"
    model, gbox = build_container(scene, mask)
    K = len(model.submodules)
    out = dict(weights_dict(model))
    P = SimpleNamespace(ray_samples=32, chunk_points=1 << 20, color_space="linear", optimizer="adam", lr=1e-4,
                        encoding_lr=0.01, sigma_lr=0.002, color_lr=0.002, bg_lr=0.001, weight_decay=0.0)
    opt = get_optimizer(P, model)
    rays, valid, _ = val_rays(scene, mask, 0.25)
    rv = rays[valid]
    g = torch.Generator().manual_seed(11)
    rows_g = torch.Generator().manual_seed(12)
    sample_rows = torch.randint(0, 16 << 20, (K, 4096), generator=rows_g)
    out["train:rows"] = _np(sample_rows)
    model.train()
    real_rand_like = torch.rand_like
    for step in range(2):
        perm = torch.randperm(rv.shape[0], generator=g)[:256]
        r = rv[perm].contiguous()
        rgbs = torch.rand(256, 3, generator=g)
        u = torch.rand(256, 32, generator=g)
        torch.rand_like = lambda t, *a, **k: u.clone() if tuple(t.shape) == tuple(u.shape) else real_rand_like(t, *a, **k)
        try:
            opt.zero_grad()
            loss = compute_mse_loss(P, model=model, data={"rays": r, "rgbs": rgbs}, params=None, active_module=None,
                                    reduction="mean")
            loss.backward()
        finally:
            torch.rand_like = real_rand_like
        pre = f"train{step}:"
        out[pre + "rays"] = _np(r); out[pre + "rgbs"] = _np(rgbs); out[pre + "u"] = _np(u)
        out[pre + "loss"] = np.array(float(loss.detach()), np.float64)
        for name, prm in model.named_parameters():
            if prm.grad is None:
                continue
            if name.endswith("hash_table"):
                k = int(name.split(".")[1])
                gt = prm.grad.detach()
                out[pre + f"grad_rows:{k}"] = _np(gt[sample_rows[k]])
                lv = gt.view(16, -1)
                out[pre + f"grad_level_sum:{k}"] = _np(lv.double().sum(1))
                out[pre + f"grad_level_sumsq:{k}"] = _np((lv.double() ** 2).sum(1))
                out[pre + f"grad_nnz:{k}"] = np.array(int((gt != 0).sum()), np.int64)
            else:
                out[pre + "grad:" + name] = _np(prm.grad)
        total = torch.nn.utils.clip_grad_norm_(model.parameters(), 1.0)
        out[pre + "total_norm"] = np.array(float(total), np.float64)
        opt.step()
        for name, prm in model.named_parameters():
            if name.endswith("hash_table"):
                k = int(name.split(".")[1])
                out[pre + f"table_rows:{k}"] = _np(prm.detach()[sample_rows[k]])
            else:
                out[pre + "param:" + name] = _np(prm)
    out["table_seeds"] = np.array([100 + k for k in range(K)], np.int64)
    out["table_scale"] = np.array(TABLE_SCALE, np.float64)
    save("train_k4", **out)


# ----------------------------------------------------------------------------------------------
OCC_RES, OCC_LEVELS, OCC_PCT, OCC_SEED0 = 32, 2, 50, 7


def occ_conf_fixture() -> dict:
    """nerf_runner.py:124-147 occupancy config at a fixture-sized grid (32^3 x 2 levels)."""
    return {"use_occ": True, "resolution": OCC_RES, "levels": OCC_LEVELS, "render_step_size": None,
            "occ_thre": 1e-2, "alpha_thre": 1e-2, "alpha_thre_start": 0.0, "alpha_thre_end": 1e-2,
            "cosine_anneal": True, "warmup_steps": 256, "update_interval": 16, "ema_decay": 0.95,
            "cone_angle": 0.004, "near_plane": 0.05, "far_plane": 1e3, "occ_frozen": False, "occ_ready": True}


def gen_occ(scene: dict) -> None:
    """Occupancy renderer fixtures: the reference's render_expert_occ / render_rays_occ /
    occupancy_marching / _merge_segments_union run over the nerfacc stand-in (_refstubs.py), with
    formula occupancy grids (oracle/occ_ref.formula_binaries, seed OCC_SEED0 + k, OCC_PCT %)."""
    from nerfs import ray_rendering as RR
    from oracle import occ_ref as R
    for mask, tag in (("g11_grid_bm110_ss11", "k1"), ("g22_grid_bm110_ss11", "k4")):
        model, gbox = build_container(scene, mask, occ_conf=occ_conf_fixture())
        K = len(model.submodules)
        with torch.no_grad():  # denser field (sigma ~ e^2.5): per-sample alpha ~1e-2, rays mostly opaque
            for sub in model.submodules:
                sub.sigma_head.bias.fill_(2.5)
        out = {}
        for k, sub in enumerate(model.submodules):
            b = R.formula_binaries(OCC_LEVELS, OCC_RES, OCC_SEED0 + k, OCC_PCT)
            with torch.no_grad():
                sub.occ_grid.binaries.copy_(torch.from_numpy(b))
                sub.occ_grid.occs.copy_(torch.from_numpy(b.reshape(-1).astype(np.float32) * 0.05))
            out[f"expert{k}:render_step_size"] = np.array(sub.render_step_size, np.float64)
            out[f"expert{k}:aabbs"] = _np(sub.occ_grid.aabbs)
        out.update(weights_dict(model))
        rays, valid, cam = val_rays(scene, mask, 0.25)
        rv = rays[valid]
        perm = torch.randperm(rv.shape[0], generator=torch.Generator().manual_seed(5))[:256]
        r = rv[perm].contiguous()
        out["rays"] = _np(r)
        sub0 = model.submodules[0]
        with torch.no_grad():
            ri, t0, t1 = sub0.occupancy_marching(r)
            out.update({"march0:ri": _np(ri), "march0:t0": _np(t0), "march0:t1": _np(t1)})
            res = RR.render_rays(model, r, ray_samples=64, active_module=0, bg_color_default="white")
            for nm, v in zip(("rgb", "depth", "weights", "acc"), res):
                out[f"expert0:{nm}"] = _np(v)
        # training-mode marching: stratified jitter (recorded) + density visibility filter
        sub0.train()
        torch.manual_seed(11)
        with torch.no_grad():
            ri, t0, t1 = sub0.occupancy_marching(r)
        sub0.eval()
        out.update({"train0:u": _np(sub0.occ_grid.last_u), "train0:ri": _np(ri), "train0:t0": _np(t0),
                    "train0:t1": _np(t1), "train0:alpha_thre": np.array(sub0.alpha_thre, np.float64)})
        if K > 1:
            # per-expert prefilter + marching lists (global ray ids) and their boundary union
            lists = ([], [], [])
            for k, sub in enumerate(model.submodules):
                hit = RR._intersect_rays_aabb(r, scene_box=sub.scene_box)
                out[f"hit{k}"] = _np(hit)
                if not hit.any():
                    continue
                with torch.no_grad():
                    ri_k, t0_k, t1_k = sub.occupancy_marching(r[hit])
                gidx = hit.nonzero(as_tuple=False).squeeze(1)[ri_k]
                lists[0].append(gidx); lists[1].append(t0_k); lists[2].append(t1_k)
                out.update({f"list{k}:ri": _np(gidx), f"list{k}:t0": _np(t0_k), f"list{k}:t1": _np(t1_k)})
            mri, m0, m1 = RR._merge_segments_union(*lists)
            out.update({"union:ri": _np(mri), "union:t0": _np(m0), "union:t1": _np(m1)})
            # container render: the reference routes x_mid.view(1, -1, 3), which its own _routing
            # asserts against (meta_container.py:111); the fixture routes the (M, 3) points
            orig = type(model)._routing

            def routing_flat(self, pts, _orig=orig):
                return _orig(self, pts.reshape(-1, 3))
            type(model)._routing = routing_flat
            try:
                with torch.no_grad():
                    res = RR.render_rays(model, r, ray_samples=64, active_module=None, bg_color_default="white")
            finally:
                type(model)._routing = orig
            for nm, v in zip(("rgb", "depth", "weights", "acc"), res):
                out[f"container:{nm}"] = _np(v)
        out["table_seeds"] = np.array([100 + k for k in range(K)], np.int64)
        out["table_scale"] = np.array(TABLE_SCALE, np.float64)
        out["bm"] = np.array(model.boundary_margin, np.float64)
        out["occ"] = np.array([OCC_RES, OCC_LEVELS, OCC_PCT, OCC_SEED0], np.int64)
        save(f"occ_{tag}", **out)
        del model


# ----------------------------------------------------------------------------------------------
class _StubLogger:
    """Logger surface train_step calls (utils.Logger writes tensorboard/files; not needed here)."""

    def log(self, *a, **k):
        pass

    def log_dirname(self, *a, **k):
        pass

    def scalar_summary(self, *a, **k):
        pass


META_S, META_RAYS, META_REGIONS = 16, 64, (0, 2)


def gen_meta(scene: dict) -> None:
    """SURVEY §8(f) rank 2 fixture: one offline meta-training step (pipelines/offline_stage/
    meta_train_step.py:18-253 train_step -> meta_core.task_adapt / meta_update) of the K=4
    container for FOMAML, second-order MAML and Reptile: 2 regions x 1 task, 64 support + 64 query
    rays x 16 samples, 2 inner steps; the training-mode jitter of every render call is recorded in
    call order (ray_rendering.py:286 draws it with torch.rand_like).  Also task_adapt alone (fast
    weights after the inner loop)."""
    import random
    from types import SimpleNamespace
    from common.utils import get_optimizer
    from pipelines.offline_stage import meta_core as MC
    from pipelines.offline_stage.meta_train_step import train_step
    from utils import MetricLogger
    mask = "g22_grid_bm110_ss11"
    rays, valid, _ = val_rays(scene, mask, 0.25)
    rv = rays[valid]
    S = META_S
    rows_g = torch.Generator().manual_seed(22)
    sample_rows = torch.randint(0, 16 << 20, (4, 2048), generator=rows_g)
    for algo in ("fomaml", "maml", "reptile"):
        model, gbox = build_container(scene, mask)
        out = dict(weights_dict(model))
        out["rows"] = _np(sample_rows)
        P = SimpleNamespace(algo=algo, ray_samples=S, chunk_points=1 << 20, color_space="linear", optimizer="adam",
                            lr=1e-4, encoding_lr=0.01, sigma_lr=0.002, color_lr=0.002, bg_lr=0.001, weight_decay=0.0,
                            inner_lr=0.05, inner_iter=2, fim=False, use_amp=False, grad_clip=1.0, seed=0,
                            mixed_precision=False, print_step=10 ** 9)
        opt = get_optimizer(P, model)
        g = torch.Generator().manual_seed(21)
        task_data = {}
        for cid in META_REGIONS:
            task = {}
            for part in ("support", "query"):
                perm = torch.randperm(rv.shape[0], generator=g)[:META_RAYS]
                task[part] = {"rays": rv[perm].contiguous(), "rgbs": torch.rand(META_RAYS, 3, generator=g)}
                out[f"task{cid}:{part}:rays"] = _np(task[part]["rays"])
                out[f"task{cid}:{part}:rgbs"] = _np(task[part]["rgbs"])
            task_data[cid] = [task]
        gu = torch.Generator().manual_seed(23)
        us = []
        real = torch.rand_like

        def fake(t, *a, **k):
            if t.dim() == 2 and t.shape[1] == S:
                u = torch.rand(tuple(t.shape), generator=gu)
                us.append(u)
                return u.clone()
            return real(t, *a, **k)
        model.train()
        torch.rand_like = fake
        try:
            if algo == "maml":  # the inner loop alone: fast weights after 2 create_graph steps
                fast, inner = MC.task_adapt(P, model, task_data[0][0]["support"], P.inner_lr, P.inner_iter,
                                            active_module=0)
                for name, v in fast.items():
                    out["adapt_fast:" + name] = _np(v)
                out["adapt_inner_losses"] = np.array([float(x) for x in inner], np.float64)
                out["adapt_n_u"] = np.array(len(us), np.int64)
            if algo != "reptile":
                train_step(P, 1, model, opt, task_data, MetricLogger(delimiter="  "), _StubLogger())
            else:
                # the reference's train_step calls meta_update without fast_list (meta_train_step.py:168),
                # so Reptile raises there; its update rule (meta_core.py:145-182) is pinned directly, with
                # the expert-relative fast names prefixed to the container's meta-parameter names
                # (unprefixed, `name in sum_delta` never matches and the update is a no-op)
                order = list(META_REGIONS)
                random.Random(P.seed + 1).shuffle(order)
                fast_list = []
                for cid in order:
                    fast, _ = MC.task_adapt(P, model, task_data[cid][0]["support"], P.inner_lr, P.inner_iter,
                                            active_module=cid)
                    fast_list.append({f"submodules.{cid}.{n}": v for n, v in fast.items()})
                MC.reptile_meta_update(P, model, fast_list)
        finally:
            torch.rand_like = real
        out["u"] = _np(torch.stack(us, 0))
        order = list(META_REGIONS)
        random.Random(P.seed + 1).shuffle(order)
        out["region_order"] = np.array(order, np.int64)
        for name, prm in model.named_parameters():
            if name.endswith("hash_table"):
                k = int(name.split(".")[1])
                out[f"after_table_rows:{k}"] = _np(prm.detach()[sample_rows[k]])
                if prm.grad is not None:
                    out[f"grad_table_rows:{k}"] = _np(prm.grad[sample_rows[k]])
            else:
                out["after:" + name] = _np(prm)
                if prm.grad is not None:
                    out["grad:" + name] = _np(prm.grad)
        out["table_seeds"] = np.array([100 + k for k in range(4)], np.int64)
        out["table_scale"] = np.array(TABLE_SCALE, np.float64)
        save(f"meta_{algo}", **out)
        del model

DATA_STEMS = ["000006", "000007", "000009", "000010"]
DATA_SCALE = 0.125
DATA_MASKS = "g22_grid_bm110_ss11"
TASK_CASES = {
    # name: (region, TaskDataset kwargs) -- "runner" is nerf_runner.py:193-201's configuration
    "runner": (0, dict(S_target=512, Q_target=256, min_rays_cell=384, image_cap=0.4, assignment_checkpoint=0.7,
                       routing_policy="dda", cells=(1, 5, 5), seed=0)),
    "alpha_box": (0, dict(S_target=400, Q_target=200, min_rays_cell=600, image_cap=None, routing_policy="alpha",
                          max_images_support=2, max_images_query=1,
                          cells=(1, 6, 6), seed=3, region_box=True)),
    "small_alpha": (2, dict(S_target=300, Q_target=150, min_rays_cell=200, image_cap=0.4, routing_policy="alpha",
                            cells=(2, 3, 3), seed=7, max_images_query=1, min_images_support=3)),
}
TASK_EPISODES = 4


def _digest(t: torch.Tensor) -> str:
    import hashlib
    return hashlib.sha256(np.ascontiguousarray(_np(t)).tobytes()).hexdigest()


def gen_data(scene: dict) -> None:
    """RamRaysDataset (per-region masks, expert box, near/far override) over 4 train images, then
    TaskDataset bins + episodes for three configurations (data/ram_rays_dataset.py, task_dataset.py)."""
    from zipfile import ZipFile
    from data.dataset import get_image_metadata as ref_get_image_metadata
    from data.ram_rays_dataset import RamRaysDataset
    from data.task_dataset import TaskDataset

    m = scene["masks"][DATA_MASKS] if DATA_MASKS in scene["masks"] else None
    b = torch.load(DATA / "masks" / DATA_MASKS / "scene_boxes.pt", map_location="cpu", weights_only=True)
    boxes = [SceneBox(aabb=torch.stack([b["mins"][k].float(), b["maxs"][k].float()])) for k in range(len(b["mins"]))]
    out = {"stems": np.array(DATA_STEMS), "scale": np.array(DATA_SCALE, np.float64),
           "box_aabbs": np.stack([_np(bx.aabb) for bx in boxes])}
    overrides = {0: (0.0, 100000.0), 2: (0.05, 1.2)}
    datasets = {}
    for region in (0, 2):
        tr, _ = ref_get_image_metadata(DATA, DATA_SCALE, DATA / "masks" / DATA_MASKS / str(region))
        items = [md for md in tr if md is not None and md.image_path.stem in DATA_STEMS]
        items.sort(key=lambda md: md.image_path.stem)
        assert len(items) == len(DATA_STEMS)
        if region == 0:
            out["images"] = np.stack([md.load_image().numpy() for md in items])
            out["c2w"] = np.stack([_np(md.c2w.float()) for md in items])
            out["intrinsics"] = np.stack([_np(md.intrinsics.float()) for md in items])
            out["image_index"] = np.array([md.image_index for md in items], np.int64)
            out["HW"] = np.array([items[0].H, items[0].W], np.int64)
        masks = []
        for md in items:
            with ZipFile(md.mask_path, "r") as zf, zf.open(zf.namelist()[0]) as f:
                mk = torch.load(f, map_location="cpu", weights_only=True)
            masks.append(np.packbits(_np(mk.bool()).reshape(-1)))
        out[f"r{region}_mask_shape"] = np.array(mk.shape, np.int64)
        out[f"r{region}_masks"] = np.stack(masks)
        ds = RamRaysDataset(items, center_pixels=True,
                            ray_gen_kwargs={"scene_box": boxes[region], "near_far_override": overrides[region]},
                            num_workers=1)
        out[f"r{region}_override"] = np.array(overrides[region], np.float64)
        out[f"r{region}_n"] = np.array(len(ds), np.int64)
        for key, t in (("rays", ds._rays), ("rgbs", ds._rgbs), ("img", ds._img_indices)):
            out[f"r{region}_{key}_sha"] = np.array(_digest(t))
        out[f"r{region}_rays_sample"] = _np(ds._rays[::61])
        out[f"r{region}_rgbs_sample"] = _np(ds._rgbs[::61])
        out[f"r{region}_img"] = _np(ds._img_indices)
        datasets[region] = ds
    for name, (region, kw) in TASK_CASES.items():
        kw = dict(kw)
        if kw.pop("region_box", False):
            kw["region_bounds"] = tuple(tuple(float(v) for v in row) for row in boxes[region].aabb.tolist())
        ds = datasets[region]
        td = TaskDataset(ds, cell_id=region, **kw)
        nv = int(td._region_segment(ds._rays, td.aabb)[0].sum())
        counts = np.array([int(x.numel()) for x in td._cell_flat_idx], np.int64)
        # bins in routing order = the flat pools un-permuted is not recoverable; store the pools
        out[f"t_{name}_n_valid"] = np.array(nv, np.int64)
        out[f"t_{name}_aabb"] = _np(td.aabb)
        out[f"t_{name}_counts"] = counts
        out[f"t_{name}_flat_idx"] = np.concatenate([_np(x) for x in td._cell_flat_idx]).astype(np.int64)
        out[f"t_{name}_eligible"] = np.array(td.eligible_cells, np.int64)
        it = iter(td)
        ep_s, ep_q, ep_meta = [], [], []
        for _ in range(TASK_EPISODES):
            task = next(it)
            ep_s.append(_np(task.support["idx"])); ep_q.append(_np(task.query["idx"]))
            ep_meta.append([task.block_id, len(ep_s[-1]), len(ep_q[-1]), int(task.metrics["image_disjoint_ok"]),
                            len(task.warnings)])
        out[f"t_{name}_support"] = np.concatenate(ep_s).astype(np.int64)
        out[f"t_{name}_query"] = np.concatenate(ep_q).astype(np.int64)
        out[f"t_{name}_episodes"] = np.array(ep_meta, np.int64)
        print(name, "valid", nv, "cells", counts.tolist(), "episodes", ep_meta)
    save("data_tasks", **out)


CLUSTER_ROUTE_CASES = {
    # name: (image index in train+val metadata order, centroid set, cluster_2d, boundary_margin, samples)
    "c2d_bm105": (0, "cent_grid22_2d", True, 1.05, 48),
    "c2d_strict": (7, "cent_grid42_2d", True, 1.0, 32),
    "c3d_bm110": (5, "cent_grid222_3d", False, 1.1, 40),
}
CLUSTER_MAIN_CASES = {
    "grid_orig": dict(centroid_mode="grid", grid_dim=[2, 2], cluster_2d=True, boundary_margin=1.05, ray_samples=32,
                      near=None, far=None, box_margin=0.0),
    "kmeans_near_far": dict(centroid_mode="kmeans", grid_dim=[2, 2], cluster_2d=True, boundary_margin=1.0,
                            ray_samples=24, near=1.0, far=200.0, box_margin=3.0, kmeans_weight_by_pixels=True),
    "grid3d": dict(centroid_mode="grid", grid_dim=[2, 1, 2], cluster_2d=False, boundary_margin=1.1, ray_samples=16,
                   near=None, far=150.0, box_margin=0.0),
}
CLUSTER_MAIN_STEMS = {"train": ["000001", "000005", "000009"], "val": ["000000"]}
CLUSTER_MAIN_SCALE = 1.0 / 32.0


def _cluster_module():
    import importlib.util
    spec = importlib.util.spec_from_file_location("ref_create_clusters", REF / "scripts" / "create_clusters.py")
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def gen_clusters(scene: dict) -> None:
    """scripts/create_clusters.py on the CPU: centroid generators, compute_voronoi_orig on three images,
    main() end to end (--orig; the CPU path) on a 4-image dataset at 1/32 resolution, plus the
    reference's own GPU-made outputs that ship with the example dataset (scene boxes, two images'
    masks) for the full-scale check on the GPU."""
    import types
    import zipfile
    from nerfs.ray_sampling import clamp_rays_near_far, get_ray_directions, get_rays
    cc = _cluster_module()
    coord = torch.load(DATA / "coordinates.pt", map_location="cpu", weights_only=True)
    metas = sorted((DATA / "train" / "metadata").glob("*.pt")) + sorted((DATA / "val" / "metadata").glob("*.pt"))
    mds = [torch.load(p, map_location="cpu", weights_only=True) for p in metas]
    out = {"meta_split": np.array([p.parent.parent.name for p in metas]), "meta_stem": np.array([p.stem for p in metas]),
           "meta_c2w": np.stack([_np(m["c2w"]) for m in mds]).astype(np.float32),
           "meta_intr": np.stack([_np(m["intrinsics"]) for m in mds]).astype(np.float64),
           "meta_HW": np.array([[int(m["H"]), int(m["W"])] for m in mds], np.int64),
           "pose_scale": np.array(float(coord["pose_scale_factor"]), np.float64),
           "origin_drb": _np(coord["origin_drb"]).astype(np.float32),
           "altitude_range_enu": _np(torch.as_tensor(coord["altitude_range_enu"])).astype(np.float64)}
    assert all(m["c2w"].dtype == torch.float32 for m in mds)
    cams = torch.stack([m["c2w"] for m in mds]).float()[..., :3, 3]
    out["cent_grid22_2d"] = _np(cc._grid_centroids(cams, 1, 2, 2, True))
    out["cent_grid42_2d"] = _np(cc._grid_centroids(cams, 1, 4, 2, True))
    out["cent_grid222_3d"] = _np(cc._grid_centroids(cams, 2, 2, 2, False))
    out["cent_km4_pp"] = _np(cc._run_kmeans(cams[:, 1:].cpu(), 4, 50, "kmeans++", 0, None))
    w = cc._cam_weights(metas)
    out["cent_km4_pp_w"] = _np(cc._run_kmeans(cams[:, 1:].cpu(), 4, 50, "kmeans++", 0, w))
    out["cent_km3_rand_3d"] = _np(cc._run_kmeans(cams.cpu(), 3, 20, "random", 5, None))
    # the global box of main() (create_clusters.py:650-700) with scene_scale 1.1, pad 10 m
    ps, ox = float(coord["pose_scale_factor"]), float(coord["origin_drb"][0])
    lo_m, hi_m = map(float, coord["altitude_range_enu"])
    gbox = SceneBox.from_bound(torch.tensor([[(-hi_m - ox) / ps, -1.1, -1.1], [(-lo_m - ox) / ps, 1.1, 1.1]],
                                            dtype=torch.float32)).expand(torch.tensor([[10.0 / ps, 0, 0]]))
    out["route_gbox"] = _np(gbox.aabb)
    for name, (idx, cset, c2d, bm, S) in CLUSTER_ROUTE_CASES.items():
        md = mds[idx]
        H, W = int(md["H"]) // 16, int(md["W"]) // 16
        fx, fy, cx, cy = [float(v) for v in (md["intrinsics"].float() / 16)]
        dirs = get_ray_directions(H, W, fx, fy, cx, cy, True, torch.device("cpu"))
        rays = get_rays(dirs, md["c2w"], scene_box=gbox, aabb_max_bound=1e10, aabb_invalid_value=float("inf")).view(-1, 8)
        rays, valid = clamp_rays_near_far(rays, (None, None))
        mask = cc.compute_voronoi_orig(rays, ray_samples=S, ray_chunk_size=4096, sample_chunk_size=S * 1000,
                                       centroids=torch.from_numpy(out[cset]), cluster_2d=c2d,
                                       device=torch.device("cpu"), boundary_margin=bm)
        out[f"route_{name}_rays_sha"] = np.array(__import__("hashlib").sha256(_np(rays).tobytes()).hexdigest())
        out[f"route_{name}_hw_intr"] = np.array([H, W, fx, fy, cx, cy], np.float64)
        out[f"route_{name}_valid"] = _np(valid)
        out[f"route_{name}_mask"] = np.packbits(_np(mask).reshape(-1))
        print(name, H, W, "valid", int(valid.sum()), "mask per centroid", _np(mask).sum(0).tolist())
    # main() end to end on a small dataset
    import shutil
    import tempfile
    root = Path(tempfile.mkdtemp(prefix="acn_cc_"))
    try:
        torch.save(dict(coord), root / "coordinates.pt")
        for split, stems in CLUSTER_MAIN_STEMS.items():
            (root / split / "metadata").mkdir(parents=True)
            for stem in stems:
                md = dict(torch.load(DATA / split / "metadata" / f"{stem}.pt", map_location="cpu", weights_only=True))
                md["H"], md["W"] = int(md["H"] * CLUSTER_MAIN_SCALE), int(md["W"] * CLUSTER_MAIN_SCALE)
                md["intrinsics"] = md["intrinsics"] * CLUSTER_MAIN_SCALE
                torch.save(md, root / split / "metadata" / f"{stem}.pt")
        out["main_stems"] = np.array([f"{sp}/{s}" for sp, ss in CLUSTER_MAIN_STEMS.items() for s in ss])
        for case, kw in CLUSTER_MAIN_CASES.items():
            h = types.SimpleNamespace(data_path=root, output=Path(case), segmentation_path=None, resume=False,
                                      kmeans_iters=50, kmeans_init="kmeans++", kmeans_seed=0,
                                      kmeans_weight_by_pixels=False, center_pixels=True, orig=True,
                                      ray_chunk_size=8192, sample_chunk_size=1 << 20, fp16=False, scene_scale=1.1,
                                      altitude_range=None, altitude_pad=10.0)
            for k_, v_ in kw.items():
                setattr(h, k_, v_)
            cc.main(h)
            od = root / "masks" / case
            params = torch.load(od / "params.pt", map_location="cpu", weights_only=True)
            boxes = torch.load(od / "scene_boxes.pt", map_location="cpu", weights_only=True)
            out[f"main_{case}_centroids"] = _np(params["centroids"])
            out[f"main_{case}_aabb_global"] = _np(boxes["aabb_global"])
            out[f"main_{case}_mins"] = _np(boxes["mins"])
            out[f"main_{case}_maxs"] = _np(boxes["maxs"])
            out[f"main_{case}_counts"] = _np(boxes["counts"])
            out[f"main_{case}_params_json"] = np.array(json.dumps(
                {k_: (list(v_) if isinstance(v_, tuple) else v_) for k_, v_ in params.items()
                 if not isinstance(v_, torch.Tensor)}))
            C_ = params["centroids"].shape[0]
            masks = []
            for sp_stem in out["main_stems"]:
                stem = str(sp_stem).split("/")[1]
                for c in range(C_):
                    with zipfile.ZipFile(od / str(c) / f"{stem}.pt") as zf, zf.open(zf.namelist()[0]) as f:
                        m = torch.load(f, map_location="cpu", weights_only=True)
                    masks.append(np.packbits(_np(m).reshape(-1)))
            out[f"main_{case}_masks"] = np.stack(masks)
            print(case, "boxes", _np(boxes["mins"]).round(4).tolist(), "counts", _np(boxes["counts"]).tolist())
    finally:
        shutil.rmtree(root, ignore_errors=True)
    # the reference's GPU-made mask sets that ship with the example dataset
    for mset in ("g22_grid_bm110_ss11", "g32_grid_bm110_ss11", "g12_grid_bm110_ss11", "g11_grid_bm110_ss11"):
        b = torch.load(DATA / "masks" / mset / "scene_boxes.pt", map_location="cpu", weights_only=True)
        p = torch.load(DATA / "masks" / mset / "params.pt", map_location="cpu", weights_only=True)
        for key in ("mins", "maxs", "counts", "centroids", "aabb_global"):
            out[f"ship_{mset}_{key}"] = _np(b[key])
        out[f"ship_{mset}_params_json"] = np.array(json.dumps(
            {k_: (list(v_) if isinstance(v_, tuple) else v_) for k_, v_ in p.items() if not isinstance(v_, torch.Tensor)}))
    for stem in ("000000", "000007"):
        for c in range(4):
            with zipfile.ZipFile(DATA / "masks" / "g22_grid_bm110_ss11" / str(c) / f"{stem}.pt") as zf, \
                    zf.open(zf.namelist()[0]) as f:
                m = torch.load(f, map_location="cpu", weights_only=True)
            out[f"ship_mask_{stem}_{c}"] = np.packbits(_np(m.bool()).reshape(-1))
    save("clusters", **out)


def main() -> None:
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    scene = scene_json()
    (HERE / "scene_drz_example.json").write_text(json.dumps(scene, indent=1))
    print("wrote scene_drz_example.json")
    which = sys.argv[1:] or ["hashgrid", "sh", "volume_render", "routing", "rays", "render", "train", "occ", "meta", "data", "clusters"]
    if "hashgrid" in which: gen_hashgrid()
    if "sh" in which: gen_sh()
    if "volume_render" in which: gen_volume_render()
    if "routing" in which: gen_routing(scene)
    if "rays" in which: gen_rays(scene)
    if "render" in which: gen_field_and_render(scene)
    if "train" in which: gen_train(scene)
    if "k8" in which: gen_k8(scene)
    if "train_k8" in which: gen_train_k8(scene)
    if "occ" in which: gen_occ(scene)
    if "meta" in which: gen_meta(scene)
    if "data" in which: gen_data(scene)
    if "clusters" in which: gen_clusters(scene)


if __name__ == "__main__":
    main()
