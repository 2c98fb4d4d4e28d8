"""Work expansion of the routed render (C3 / C4) on the CPU, from the oracle's routing.

For the bench's C3 batch (4096 random valid pixels of validation camera 0, 256 samples, g22 soft
routing bm 1.05, rays sorted by the expert owning their midpoint) it counts
  * (sample, expert) pairs per sample  -- the work the reference's expert loop does,
  * expert evaluations per sample when a 32-sample tile evaluates every expert any of its samples
    needs (render_kernel / render_slots_kernel: one wave-uniform decision per tile),
  * rays whose experts are not all among the two a slots-kernel workgroup stages.
Usage: python tools/route_stats.py [--k 4|8] [--rays 4096] [--samples 256] [--wg 8]
"""
import argparse
import json
import sys
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))
from oracle import oracle as O  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--k", type=int, default=4)
    ap.add_argument("--rays", type=int, default=4096)
    ap.add_argument("--samples", type=int, default=256)
    ap.add_argument("--wg", type=int, default=8, help="rays per slots-kernel workgroup round")
    a = ap.parse_args()
    scene = json.loads((REPO / "tests" / "golden" / "scene_drz_example.json").read_text())
    if a.k == 4:
        sc = scene["masks"]["g22_grid_bm110_ss11"]
    else:
        import torch  # noqa: F401  (synthetic.grid_layout is plain python)
        from adaptive_city_nerf_amd.synthetic import grid_layout
        sc = grid_layout(4, 2, scene)
    cam = scene["val_cam0"]
    ds = 0.25
    H, W = int(round(cam["H"] * ds)), int(round(cam["W"] * ds))
    intr = [v * ds for v in cam["intrinsics"]]
    psf = scene["pose_scale_factor"]
    rays, valid = O.get_rays(H, W, *intr, np.asarray(cam["c2w"], np.float32), np.asarray(sc["aabb_global"], np.float32),
                             near_far_override=(0.0 / psf, 100000 / psf))
    import torch
    vi = torch.nonzero(torch.from_numpy(valid)).squeeze(1)
    g = torch.Generator().manual_seed(1234)
    sel = vi[torch.randperm(vi.numel(), generator=g)[: a.rays]].numpy()
    rays = rays[sel]
    N, S = rays.shape[0], a.samples
    cent = np.asarray(sc["centroids"], np.float32)
    K = cent.shape[0]
    bm = min(max(1.0, 1.05), sc["boundary_margin"])
    # dominant expert of the midpoint (parallel.dominant_expert), stable sort
    near, far = rays[:, 6], rays[:, 7]
    mid = np.where(np.isfinite(far), 0.5 * (near + far), 0.0).astype(np.float32)
    mid = np.where(np.isfinite(mid), mid, 0.0).astype(np.float32)
    _, hard = O.routing(rays[:, :3] + rays[:, 3:6] * mid[:, None], cent, sc["cluster_2d"], 1.0)
    order = np.argsort(hard, kind="stable")
    rays = rays[order]
    step = np.float32(1.0) / np.float32(S - 1)
    u = np.arange(S, dtype=np.float32) * step
    t = rays[:, 6:7] * (1 - u) + rays[:, 7:8] * u
    pts = rays[:, None, :3] + rays[:, None, 3:6] * t[..., None]
    Wr, _ = O.routing(pts.reshape(-1, 3), cent, sc["cluster_2d"], bm)
    need = (Wr > 0).reshape(N, S, K)
    pairs = need.sum(-1)
    T = (S + 31) // 32
    tiles = np.zeros((N, T, K), bool)
    for ti in range(T):
        tiles[:, ti] = need[:, ti * 32:(ti + 1) * 32].any(1)
    evals = tiles.sum(-1) * np.minimum(32, S - 32 * np.arange(T))[None]
    raymask = need.any(1)
    out = {"K": K, "rays": N, "samples": S,
           "pairs_per_sample": float(pairs.mean()),
           "samples_by_experts": {int(c): float((pairs == c).mean()) for c in range(K + 1)},
           "tile_evals_per_sample": float(evals.sum() / (N * S)),
           "tiles_multi_expert": float((tiles.sum(-1) > 1).mean()),
           "experts_per_ray": float(raymask.sum(-1).mean())}
    # workgroup rounds of `wg` consecutive sorted rays: the two most needed experts staged
    miss = 0
    unions = []
    for b in range(0, N, a.wg):
        m = raymask[b:b + a.wg]
        cnt = m.sum(0)
        top = np.argsort(-cnt, kind="stable")[:2]
        res = np.zeros(K, bool); res[top[cnt[top] > 0]] = True
        miss += int((m & ~res).any(1).sum())
        unions.append(int(m.any(0).sum()))
    out["rays_with_nonresident_expert"] = miss / N
    out["experts_per_round_union"] = float(np.mean(unions))
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
