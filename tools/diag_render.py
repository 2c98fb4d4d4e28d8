"""Diagnostic: in-kernel shader clock of a render_kernel built with -DACN_DIAG_CLOCK=1 (the build
writes the per-ray clock in MHz into depth).  ACNERF_LIB=... python tools/diag_render.py"""
import sys, time
from pathlib import Path
import torch
REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO))
import bench  # noqa: E402
from adaptive_city_nerf_amd import render_rays, ops  # noqa: E402
dev = torch.device("cuda", 0)
model, gbox, scene, sc = bench.build_model(dev, 1)
rays = bench.make_rays(scene, gbox, dev, 4096, 1234)
with torch.no_grad():
    t_end = time.time() + 3.0
    n = 0
    while time.time() < t_end:
        out = render_rays(model, rays, ray_samples=256, bg_color_default="white")
        n += 1
    torch.cuda.synchronize()
    ops.EVENT_HOOK = []
    for _ in range(20):
        out = render_rays(model, rays, ray_samples=256, bg_color_default="white")
    torch.cuda.synchronize()
    ms = sum(a.elapsed_time(b) for a, b in ops.EVENT_HOOK) / len(ops.EVENT_HOOK)
d = out[1].float()
print(f"{n} warm launches; kernel {ms:.4f} ms; depth: median {d.median().item():.0f} "
      f"min {d.min().item():.0f} max {d.max().item():.0f}; acc median {out[3].float().median().item():.0f}; "
      f"rgb.r median {out[0][:, 0].float().median().item():.0f}")
