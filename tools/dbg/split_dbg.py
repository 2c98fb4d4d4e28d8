"""debug: which rays differ between the split and the unsplit routed render"""
import sys
sys.path.insert(0, "tests"); sys.path.insert(0, ".")
import numpy as np, torch
import goldens as G
from test_k8 import _model, _single_expert_rays, MASK
from adaptive_city_nerf_amd import ops, render_rays
d = G.load("render_k8")
m, _ = _model(d)
sc = G.scene()["masks"][MASK]
rays0 = torch.from_numpy(d["render:rays"]).cuda()
ks0 = _single_expert_rays(d["render:rays"], 64, sc, float(d["bm"]))
g = torch.Generator(device="cuda").manual_seed(5)
perm = torch.randperm(rays0.shape[0], device="cuda", generator=g)
for name, idx in (("orig", torch.arange(rays0.shape[0], device="cuda")), ("perm", perm)):
    rays = rays0[idx].contiguous()
    ks = ks0[idx.cpu().numpy()]
    outs = []
    for split in (True, False):
        ops.REORDER = split
        with torch.no_grad():
            outs.append([t.clone() for t in render_rays(m, rays, ray_samples=64, bg_color_default="white")])
    ops.REORDER = True
    diff = (outs[0][0] - outs[1][0]).abs().max(1).values.cpu().numpy()
    bad = np.nonzero(diff > 0)[0]
    print(name, "n bad", len(bad), "max diff", diff.max(), "classes of bad", np.unique(ks[bad], return_counts=True))
    # against active_module for expert 2's single rays
    sel = np.nonzero(ks == 2)[0]
    with torch.no_grad():
        am = render_rays(m, rays[torch.from_numpy(sel).cuda()], ray_samples=64, bg_color_default="white", active_module=2)[0]
    for split in (0, 1):
        dd = (outs[split][0][torch.from_numpy(sel).cuda()] - am).abs().max(1).values.cpu().numpy()
        print(name, "split" if split == 0 else "unsplit", "vs active_module: n diff", int((dd > 0).sum()), "max", dd.max())
