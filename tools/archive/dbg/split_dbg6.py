"""debug: determinism of render_kernel (active_module) on the single-expert subset, several orders"""
import sys
sys.path.insert(0, "tests"); sys.path.insert(0, ".")
import numpy as np, torch
import goldens as G
from test_k8 import _model, _single_expert_rays, MASK
from adaptive_city_nerf_amd import ops, render_rays
d = G.load("render_k8")
m, _ = _model(d, "hiw:")
sc = G.scene()["masks"][MASK]
rays0 = torch.from_numpy(d["render:rays"]).cuda()
ks0 = _single_expert_rays(d["render:rays"], 64, sc, float(d["bm"]))
for k in np.unique(ks0[ks0 >= 0]):
    sel = np.nonzero(ks0 == k)[0]
    sub = rays0[torch.from_numpy(sel).cuda()].contiguous()
    for reorder in (False, True):
        ops.REORDER = reorder
        with torch.no_grad():
            outs = [render_rays(m, sub, ray_samples=64, bg_color_default="white", active_module=int(k))[0].clone()
                    for _ in range(10)]
        print("expert", k, "n", len(sel), "reorder", reorder, "run-to-run max diff",
              max(float((x - outs[0]).abs().max()) for x in outs), flush=True)
    ops.REORDER = True
