"""debug: consistency of the split render's ray lists over repeated runs"""
import sys, types
sys.path.insert(0, "tests"); sys.path.insert(0, ".")
import numpy as np, torch
import goldens as G
from test_k8 import _model
from adaptive_city_nerf_amd import ops, render_rays
d = G.load("render_k8")
m, _ = _model(d)
rays0 = torch.from_numpy(d["render:rays"]).cuda()
g = torch.Generator(device="cuda").manual_seed(5)
perm = torch.randperm(rays0.shape[0], device="cuda", generator=g)
rays = rays0[perm].contiguous()
N, K = rays.shape[0], 8
captured = []
real_empty = torch.empty
class Proxy(types.ModuleType):
    def __getattr__(self, k):
        return getattr(torch, k)
px = Proxy("torchproxy")
def empty(*a, **k):
    t = real_empty(*a, **k)
    if k.get("dtype") == torch.int32 and t.dim() == 1:
        captured.append(t)
    return t
px.empty = empty
ops.torch = px
for run in range(6):
    captured.clear()
    with torch.no_grad():
        rgb = render_rays(m, rays, ray_samples=64, bg_color_default="white")[0]
    torch.cuda.synchronize()
    sc = captured[-1].cpu().numpy()
    code = sc[:N]; lst = sc[N:2 * N + 128]; multi = sc[2 * N + 128:3 * N + 128]; hdr = sc[3 * N + 128:3 * N + 128 + K + 2]
    nm = hdr[K + 1]
    singles = lst[:hdr[K]]
    got = np.concatenate([singles[singles >= 0], multi[:nm]])
    ok = np.array_equal(np.sort(got), np.arange(N))
    print("run", run, "hdr", hdr.tolist(), "multi", nm, "cover ok", ok, "codes hist", np.unique(code, return_counts=True),
          "rgb sum", float(rgb.double().sum()))
