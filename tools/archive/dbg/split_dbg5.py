"""debug: run-to-run determinism of the split routed render and its single-expert rays against the
active_module render (one library variant per process: ACNERF_LIB)"""
import os, sys
sys.path.insert(0, "tests"); sys.path.insert(0, ".")
import numpy as np, torch
import goldens as G
from test_k8 import _model, _single_expert_rays, MASK
from adaptive_city_nerf_amd import render_rays
d = G.load("render_k8")
m, _ = _model(d, "hiw:")
sc = G.scene()["masks"][MASK]
rays0 = torch.from_numpy(d["render:rays"]).cuda()
ks0 = _single_expert_rays(d["render:rays"], 64, sc, float(d["bm"]))
g = torch.Generator(device="cuda").manual_seed(5)
perm = torch.randperm(rays0.shape[0], device="cuda", generator=g)
rays = rays0[perm].contiguous()
ks = ks0[perm.cpu().numpy()]
with torch.no_grad():
    runs = [render_rays(m, rays, ray_samples=64, bg_color_default="white")[0].clone() for _ in range(10)]
det = max(float((x - runs[0]).abs().max()) for x in runs)
bad = 0
for k in np.unique(ks[ks >= 0]):
    sel = torch.from_numpy(np.nonzero(ks == k)[0]).cuda()
    with torch.no_grad():
        am = render_rays(m, rays[sel], ray_samples=64, bg_color_default="white", active_module=int(k))[0]
    for r in runs:
        bad += int(((r[sel] - am).abs().max(1).values > 0).sum())
print(os.environ.get("ACNERF_LIB", "default"), "run-to-run max diff", det, "single rays != active_module over 10 runs:", bad,
      flush=True)
