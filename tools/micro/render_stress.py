"""Run-to-run stability of the render kernels on one batch (developer diagnostic): the K = 4 fixture's rays
(4096 drawn as in tests/test_render_ws.py), S = 200 with jitter, rendered R times through the per-wave slots
path (soft routing) and the work-shared one-expert path (active_module 2); every render compared bitwise with
the first.  python tools/micro/render_stress.py [R]"""
import sys
from pathlib import Path

import numpy as np
import torch

REPO = Path(__file__).resolve().parent.parent.parent
sys.path.insert(0, str(REPO))
sys.path.insert(0, str(REPO / "tests"))
import test_render_ws as T  # noqa: E402
from adaptive_city_nerf_amd import ops  # noqa: E402

R = int(sys.argv[1]) if len(sys.argv) > 1 else 50
S, n = 200, 4096
d, specs, routing, bg = T._setup("k4")
base = T._t(d["render:rays"])
g = torch.Generator(device="cuda").manual_seed(5 + n)
idx = torch.randint(0, base.shape[0], (n,), device="cuda", generator=g)
rays = base[idx].contiguous()
jit = torch.rand(n, S, device="cuda", generator=g)
for name, active, tau in (("slots per-wave", None, 0.0), ("slots per-wave tau", None, 1e-45),
                          ("ws one-expert", 2, 0.0), ("render_kernel one-expert", 2, 1e-45)):
    ref = None
    bad_renders, bad_rays = 0, 0
    with torch.no_grad():
        for r in range(R):
            rgb = ops.render_stratified(rays, S, specs, routing, active, bg[0], tau=tau, jitter=jit)[0].cpu().numpy()
            if ref is None:
                ref = rgb
                continue
            diff = np.any(rgb != ref, axis=1)
            if diff.any():
                bad_renders += 1
                bad_rays += int(diff.sum())
    print(f"{name}: {R} renders, {bad_renders} differ from the first ({bad_rays} rays)", flush=True)
