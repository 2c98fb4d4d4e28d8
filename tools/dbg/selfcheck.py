"""Self-check builds of the fused render: every 32-sample field tile is evaluated twice and a
lane whose second evaluation differs bitwise poisons its sample (NaN rgb), so a ray with a NaN colour is a
run-to-run difference caught in the act.
  ACN_WS_CHECK=1     render_ws_kernel (one expert): the second evaluation runs colour layer 0 unfolded (SH k-step
                     first, bit for bit the per-ray fold + folded layer), so the fold is checked too
  ACN_SLOTS_CHECK=1  render_slots_kernel's per-wave path (K > 2): the second evaluation redoes every fold
Run with ACNERF_LIB=<variant .so> (tools/build_variants.sh).  Cases: the reference K = 4 fixture's rays with
active_module 2 (one expert) and soft routing, and the K = 8 fixture, 4096 rays, S = 64 / 200 / 256, eval and
training jitter, `reps` renders each."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "tests"))
import numpy as np
import torch

from test_render_ws import _setup, _t

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
from adaptive_city_nerf_amd import ops

lib = os.environ.get("ACNERF_LIB", "default")
total = 0
import ctypes
from adaptive_city_nerf_amd import _lib
L = _lib.lib()
fetch = getattr(L, "acn_debug_check_fetch", None)   # ACN_SLOTS_CHECK=2 builds: the recorded mismatches
recs = []
if fetch is not None:
    fetch.argtypes, fetch.restype = [ctypes.c_void_p, ctypes.c_int], ctypes.c_int
    buf = np.zeros((4096, 16), np.float32)
for tag, active in (("k4", 2), ("k4", None), ("k8", None)):
    d, specs, routing, bg = _setup(tag)
    base = _t(d["render:rays"])
    base = base[torch.isfinite(base[:, 6:8]).all(dim=1)]   # invalid rays render NaN by design (clamp_rays_near_far)
    for S in (64, 200, 256):
        for jitter in (False, True):
            g = torch.Generator(device="cuda").manual_seed(S + 7 * jitter)
            idx = torch.randint(0, base.shape[0], (4096,), device="cuda", generator=g)
            rays = base[idx].contiguous()
            jit = torch.rand(4096, S, device="cuda", generator=g) if jitter else None
            bad = 0
            first = None
            with torch.no_grad():
                for _ in range(reps):
                    rgb = ops.render_stratified(rays, S, specs, routing, active, bg[0], tau=0.0, jitter=jit)[0]
                    if first is None:
                        first = rgb.clone()
                    bad += int(torch.isnan(rgb).any(dim=-1).sum())
                    bad += int((~((rgb == first) | torch.isnan(rgb) | torch.isnan(first))).any(dim=-1).sum())
                    if fetch is not None:
                        torch.cuda.synchronize()
                        nrec = fetch(buf.ctypes.data, 4096)
                        for r in buf[:min(nrec, 4096)]:
                            recs.append((tag, S, jitter) + tuple(float(v) for v in r))
            total += bad
            print(f"{os.path.basename(lib)} {tag} active={active} S={S} jitter={jitter}: {bad} rays flagged "
                  f"over {reps} renders", flush=True)
print(f"{os.path.basename(lib)} TOTAL flagged: {total}", flush=True)
if recs:
    print("recorded mismatches: tag S jitter | ray sample single k_single k0 k1 | r1 r2 g1 g2 b1 b2 s1 s2 | lane folded")
    for r in recs[:200]:
        t = r[:3]
        v = r[3:]
        d = [abs(v[6] - v[7]), abs(v[8] - v[9]), abs(v[10] - v[11]), abs(v[12] - v[13]) / max(abs(v[13]), 1e-30)]
        print(t, [int(x) for x in v[:6]], "diff r/g/b/rel-sigma %.3g %.3g %.3g %.3g" % tuple(d), "lane", int(v[14]),
              "folded", int(v[15]))
