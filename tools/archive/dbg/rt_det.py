"""Routed render determinism probe: full batch vs a second run vs a permutation (per-ray bitwise).
python tools/dbg/rt_det.py   (ACNERF_LIB selects a variant build)"""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "tests"))
import numpy as np
import torch
from test_batch_independence import _setup, _render

for tag, prefix in (("k4", "w:"), ("k8", "w:")):
    d, specs, routing, bg = _setup(tag, prefix, None)
    rays = torch.from_numpy(np.ascontiguousarray(d["render:rays"])).cuda()
    n = rays.shape[0]
    g = torch.Generator(device="cuda").manual_seed(17)
    perm = torch.randperm(n, device="cuda", generator=g)
    with torch.no_grad():
        a = _render(rays, None, specs, routing, bg, 0.0, 64)
        b = _render(rays, None, specs, routing, bg, 0.0, 64)
        c = _render(rays[perm].contiguous(), None, specs, routing, bg, 0.0, 64)
    for name, o in (("rerun", b), ("perm", [x[perm] for x in a])):
        ref = c if name == "perm" else a
        for w, x, y in zip(("rgb", "depth", "weights", "acc"), o, ref):
            x = x.cpu().numpy().reshape(n, -1); y = y.cpu().numpy().reshape(n, -1)
            bad = ~np.all((x == y) | (np.isnan(x) & np.isnan(y)), axis=1)
            print(tag, name, w, "rays differing", int(bad.sum()), "max", float(np.nanmax(np.abs(x - y))) if bad.any() else 0.0,
                  "idx", np.nonzero(bad)[0][:8].tolist(), flush=True)
    # fixture distance
    for w, x in zip(("rgb", "depth", "weights", "acc"), a):
        print(tag, "fixture", w, float(np.nanmax(np.abs(x.cpu().numpy() - d[f"render:{w}"]))))

if os.environ.get("RT_DEBUG"):
    for tag in ("k4", "k8"):
        d, specs, routing, bg = _setup(tag, "w:", None)
        rays = torch.from_numpy(np.ascontiguousarray(d["render:rays"])).cuda()
        with torch.no_grad():
            _, dep, _, acc = _render(rays, None, specs, routing, bg, 0.0, 64)
        dep = dep.cpu().numpy(); acc = acc.cpu().numpy()
        print(tag, "debug: rays with miscounted samples", int((dep > 0).sum()), "total bad samples", float(dep.sum()),
              "rays with multi-expert samples", int((acc > 0).sum()), "bad rays idx", np.nonzero(dep > 0)[0][:10].tolist(),
              "their multi counts", acc[dep > 0][:10].tolist())
