"""Does ray order change the C2 render kernel's speed?  (developer experiment)

Renders the bench batch (4096 random valid pixels x 256 samples) in three orders:
  random   -- the bench order (randperm of the valid pixels)
  sorted   -- the same rays sorted by pixel index (image rows)
  xcd      -- sorted, then permuted so that XCD x (blocks b with b % 8 == x) walks the x-th
              contiguous eighth of the sorted rays (one L2 per image band)
python tools/micro/ray_order.py
"""
import sys
from pathlib import Path

import torch

REPO = Path(__file__).resolve().parent.parent.parent
sys.path.insert(0, str(REPO))

import bench  # noqa: E402
from adaptive_city_nerf_amd import ops, render_rays  # noqa: E402


def xcd_order(n, waves_per_block=16, n_xcd=8):
    blocks = n // waves_per_block
    per_xcd = n // n_xcd
    idx = torch.empty(n, dtype=torch.long)
    for b in range(blocks):
        x, j = b % n_xcd, b // n_xcd
        base = x * per_xcd + j * waves_per_block
        idx[b * waves_per_block:(b + 1) * waves_per_block] = torch.arange(base, base + waves_per_block)
    return idx


def main():
    dev = torch.device("cuda", 0)
    model, gbox, scene, sc = bench.build_model(dev, 1)
    H, W, intr, c2w = bench.frame_camera(scene)
    psf = scene["pose_scale_factor"]
    rays_all, valid = ops.get_rays_image(H, W, *intr, c2w, gbox.aabb, dev, near_far_override=(0.0 / psf, 100000 / psf))
    vi = torch.nonzero(valid).squeeze(1).cpu()
    g = torch.Generator().manual_seed(7)
    sel = vi[torch.randperm(vi.numel(), generator=g)[:4096]]
    ssel = torch.sort(sel).values
    def morton(v):
        v = v & 1023
        v = (v | (v << 8)) & 0x00FF00FF
        v = (v | (v << 4)) & 0x0F0F0F0F
        v = (v | (v << 2)) & 0x33333333
        return (v | (v << 1)) & 0x55555555
    row, col = ssel // W, ssel % W
    zsel = ssel[torch.argsort(morton(col) | (morton(row) << 1))]
    csel = ssel[torch.argsort(col * H + row)]
    orders = {"random": (sel, False), "random+reorder": (sel, True), "rows": (ssel, False),
              "cols": (csel, False), "zorder": (zsel, False), "rows+reorder": (ssel, True)}
    times = {}
    ref = None
    for name, (s, reo) in orders.items():
        ops.REORDER = reo
        rays = rays_all[s.to(dev)].contiguous()
        with torch.no_grad():
            for _ in range(5):
                rgb, *_ = render_rays(model, rays, ray_samples=256, bg_color_default="white")
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(50):
                rgb, *_ = render_rays(model, rays, ray_samples=256, bg_color_default="white")
            e1.record()
            torch.cuda.synchronize()
        times[name] = e0.elapsed_time(e1) / 50
        # same rays, same colours, whatever the order
        back = torch.empty_like(rgb)
        pos = {int(p): i for i, p in enumerate(s.tolist())}
        perm = torch.tensor([pos[int(p)] for p in sel.tolist()], device=dev)
        back = rgb[perm]
        if ref is None:
            ref = back
        print(f"{name:15s} {times[name]:.4f} ms/call  max|rgb - random order| = {float((back - ref).abs().max()):.1e}",
              flush=True)


if __name__ == "__main__":
    main()
