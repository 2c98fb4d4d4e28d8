"""debug: determinism of the split routed render and the ray that differs"""
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
rays = rays0[perm].contiguous()
ks = ks0[perm.cpu().numpy()]
def rend(r, split):
    ops.REORDER = split
    with torch.no_grad():
        o = render_rays(m, r, ray_samples=64, bg_color_default="white")[0].clone()
    ops.REORDER = True
    return o
runs = [rend(rays, True) for _ in range(5)]
print("split run-to-run max diff", max(float((x - runs[0]).abs().max()) for x in runs))
uns = rend(rays, False)
sel = np.nonzero(ks == 2)[0]
with torch.no_grad():
    am = render_rays(m, rays[torch.from_numpy(sel).cuda()], ray_samples=64, bg_color_default="white", active_module=2)[0]
for i, r in enumerate(runs):
    dd = (r[torch.from_numpy(sel).cuda()] - am).abs().max(1).values.cpu().numpy()
    print("run", i, "n diff vs am", int((dd > 0).sum()), [int(sel[j]) for j in np.nonzero(dd > 0)[0]])
bad = [int(sel[j]) for j in np.nonzero(((runs[0][torch.from_numpy(sel).cuda()] - am).abs().max(1).values > 0).cpu().numpy())[0]]
for b in bad:
    one = rend(rays[b:b + 1].contiguous(), True)
    print("ray", b, "alone split", one.cpu().numpy(), "in batch split", runs[0][b].cpu().numpy(), "unsplit", uns[b].cpu().numpy())
# classification codes through the library: rerun split with a scratch we can read
from adaptive_city_nerf_amd import _lib
N = rays.shape[0]
obytes = int(_lib.lib().acn_render_order_bytes(N))
print("order bytes", obytes)
