"""Quick kernel-level timing of the fused render at BASELINE config C2 (developer tool).

python tools/perf_render.py [--rays 4096] [--samples 256] [--iters 20] [--experts 1]
"""
import argparse
import sys
import time
from pathlib import Path

import numpy as np
import torch

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO))
sys.path.insert(0, str(REPO / "tests"))

from adaptive_city_nerf_amd import ops  # noqa: E402
from adaptive_city_nerf_amd.synthetic import formula_table  # noqa: E402
import goldens as G  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rays", type=int, default=4096)
    ap.add_argument("--samples", type=int, default=256)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--experts", type=int, default=1)
    ap.add_argument("--tau", type=float, default=0.0)
    a = ap.parse_args()
    dev = "cuda"
    mask = "g11_grid_bm110_ss11" if a.experts == 1 else "g22_grid_bm110_ss11"
    d = G.load("render_k1" if a.experts == 1 else "render_k4")
    sc = G.scene()["masks"][mask]
    K = len(sc["centroids"])
    res = [16, 23, 33, 48, 70, 101, 147, 212, 307, 445, 645, 933, 1351, 1955, 2830, 4095]
    specs = []
    for k in range(K):
        tab = torch.from_numpy(formula_table(16, 20, 2, 100 + k, 0.5)).to(dev)
        w = {key[len(f"hiw:submodules.{k}."):]: torch.from_numpy(v).to(dev) for key, v in d.items()
             if key.startswith(f"hiw:submodules.{k}.") and key[len(f"hiw:submodules.{k}."):] in ops.MLP_SHAPES}
        specs.append(ops.ExpertSpec(tab, res, 20, 1, sc["mins"][k], d[f"w:submodules.{k}.aabb_extent"].tolist(), w))
    routing = ops.make_routing(torch.tensor(sc["centroids"]), K, True, 1.05)
    bgw = {k[len("hiw:bg_mlp."):]: torch.from_numpy(v).to(dev) for k, v in d.items() if k.startswith("hiw:bg_mlp.")}
    bg, keep = ops.make_background("mlp", mlp=bgw)
    cam = G.scene()["val_cam0"]
    intr = np.array(cam["intrinsics"], np.float32) * np.float32(0.25)
    rays_all, valid = ops.get_rays_image(384, 512, *intr.tolist(), torch.tensor(cam["c2w"]),
                                         torch.tensor(sc["aabb_global"]), dev, near_far_override=(0.0, 439.7))
    vi = torch.nonzero(valid).squeeze(1)
    g = torch.Generator().manual_seed(0)
    sel = vi[torch.randperm(vi.numel(), generator=g)[: a.rays].to(dev)]
    rays = rays_all[sel].contiguous()
    for _ in range(3):
        ops.render_stratified(rays, a.samples, specs, routing, None, bg, tau=a.tau)
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record()
    t0 = time.perf_counter()
    for _ in range(a.iters):
        ops.render_stratified(rays, a.samples, specs, routing, None, bg, tau=a.tau)
    ev1.record()
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / a.iters
    ms = ev0.elapsed_time(ev1) / a.iters
    M = a.rays * a.samples
    print(f"K={K} rays={a.rays} S={a.samples}: {ms:.3f} ms/call (events), {wall*1e3:.3f} ms wall, "
          f"{M / (ms * 1e-3):.3e} samples/s, {26880 * M / (ms * 1e-3) / 1e12:.1f} TFLOP/s algorithmic")


if __name__ == "__main__":
    main()
