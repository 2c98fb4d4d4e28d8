"""debug: split render lists vs differing rays"""
import sys, types
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
N, K, KM = rays.shape[0], 8, 16
sel = np.nonzero(ks == 2)[0]
with torch.no_grad():
    am = render_rays(m, rays[torch.from_numpy(sel).cuda()], ray_samples=64, bg_color_default="white", active_module=2)[0]
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
    scr = captured[-1].cpu().numpy()
    code = scr[:N]; lst = scr[N:2 * N + 16 * KM]; multi = scr[2 * N + 16 * KM:3 * N + 16 * KM]
    hdr = scr[3 * N + 16 * KM:3 * N + 16 * KM + KM + 2]
    nm = hdr[K + 1]
    singles = lst[:hdr[K]]
    got = np.concatenate([singles[singles >= 0], multi[:nm]])
    ok = np.array_equal(np.sort(got), np.arange(N))
    dd = (rgb[torch.from_numpy(sel).cuda()] - am).abs().max(1).values.cpu().numpy()
    bad = [int(sel[j]) for j in np.nonzero(dd > 0)[0]]
    where = ["single" if b in set(singles.tolist()) else ("multi" if b in set(multi[:nm].tolist()) else "none") for b in bad]
    pos = [int(np.nonzero(singles == b)[0][0]) if w == "single" else -1 for b, w in zip(bad, where)]
    print("run", run, "hdr", hdr[:K + 2].tolist(), "cover ok", ok, "bad", bad, where, "pos in single list", pos, flush=True)
