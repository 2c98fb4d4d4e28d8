"""Visiting order of a full frame's rays vs the routed render's time (developer tool, C4 shape).

The fused render reads hash cells through each XCD's L2; rays rendered at the same time share fine
cells only when they are image neighbours.  This times render_rays over the same 8-expert C4 frame
with the rays permuted into scanline order (what render_image hands over), square pixel tiles, and
Morton (Z) order; outputs are identical up to the permutation (checked).

python tools/frame_order.py [--frame 800] [--samples 256] [--iters 5]
"""
import argparse
import sys
from pathlib import Path

import torch

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO))
import bench  # noqa: E402
from adaptive_city_nerf_amd import ops, render_rays  # noqa: E402


def tile_order(H, W, t):
    y, x = torch.meshgrid(torch.arange(H), torch.arange(W), indexing="ij")
    key = ((y // t) * ((W + t - 1) // t) + (x // t)) * (t * t) + (y % t) * t + (x % t)
    return torch.argsort(key.reshape(-1))


def morton_order(H, W):
    y, x = torch.meshgrid(torch.arange(H), torch.arange(W), indexing="ij")
    key = torch.zeros(H, W, dtype=torch.int64)
    for b in range(12):
        key |= ((x >> b) & 1) << (2 * b)
        key |= ((y >> b) & 1) << (2 * b + 1)
    return torch.argsort(key.reshape(-1))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frame", type=int, default=800)
    ap.add_argument("--samples", type=int, default=256)
    ap.add_argument("--iters", type=int, default=5)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    model, gbox, scene, sc = bench.build_model(dev, 8)
    H, W, intr, c2w = bench.frame_camera(scene, a.frame, a.frame)
    rays, _ = ops.get_rays_image(H, W, *intr, c2w, gbox.aabb, dev, center_pixels=True,
                                 near_far_override=(None, None), apply_clamp=True)
    orders = {"scanline": torch.arange(H * W), "tile8": tile_order(H, W, 8), "tile16": tile_order(H, W, 16),
              "tile32": tile_order(H, W, 32), "morton": morton_order(H, W)}
    ref = None
    for name, perm in orders.items():
        perm = perm.to(dev)
        r = rays[perm].contiguous()
        with torch.no_grad():
            out = render_rays(model, r, ray_samples=a.samples, bg_color_default="white", _want_weights=False)[0]
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                render_rays(model, r, ray_samples=a.samples, bg_color_default="white", _want_weights=False)
            e1.record()
            torch.cuda.synchronize()
        img = torch.empty_like(out)
        img[perm] = out
        if ref is None:
            ref = img
        same = bool(torch.equal(img, ref))
        ms = e0.elapsed_time(e1) / a.iters
        print(f"{name:9s} {ms:8.3f} ms/frame  {H * W * a.samples / ms / 1e6:.3f} Gsamples/s  identical={same}",
              flush=True)


if __name__ == "__main__":
    main()
