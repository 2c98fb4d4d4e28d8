"""Run-to-run and kernel-to-kernel comparison of the single-expert render on one batch (developer diagnostic):
render_ws_kernel (tau = 0) and render_kernel (tau = 1e-45), several calls each, the failing case of
tests/test_render_ws.py (k4 fixture, active_module 2, S = 200, 4096 rays)."""
import sys
from pathlib import Path

import numpy as np
import torch

REPO = Path(__file__).resolve().parent.parent.parent
sys.path.insert(0, str(REPO))
sys.path.insert(0, str(REPO / "tests"))
import test_render_ws as T  # noqa: E402
from adaptive_city_nerf_amd import ops  # noqa: E402

tag, active, S, n = "k4", 2, int(sys.argv[1]) if len(sys.argv) > 1 else 200, 4096
d, specs, routing, bg = T._setup(tag)
base = T._t(d["render:rays"])
g = torch.Generator(device="cuda").manual_seed(5 + n)
idx = torch.randint(0, base.shape[0], (n,), device="cuda", generator=g)
rays = base[idx].contiguous()
outs = {"ws": [], "rk": []}
with torch.no_grad():
    for rep in range(4):
        for name, tau in (("ws", 0.0), ("rk", 1e-45)):
            o = ops.render_stratified(rays, S, specs, routing, active, bg[0], tau=tau)
            outs[name].append([x.cpu().numpy() for x in o])
for name in outs:
    for r in range(1, 4):
        diff = [not np.array_equal(a, b, equal_nan=True) for a, b in zip(outs[name][0], outs[name][r])]
        print(name, "call 0 vs", r, "differs (rgb, depth, weights, acc):", diff)
for r in range(4):
    a, b = outs["ws"][r], outs["rk"][r]
    bad = np.nonzero(np.any(a[0] != b[0], axis=1))[0]
    print("call", r, "ws vs rk rgb rays differing:", bad.size, bad[:8],
          "max|d|", float(np.abs(a[0] - b[0]).max()) if bad.size else 0.0)
    if bad.size:
        k = bad[0]
        print("  ray", k, "ws", a[0][k], "rk", b[0][k], "acc", a[3][k], b[3][k], "depth", a[1][k], b[1][k])
