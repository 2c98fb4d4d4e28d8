"""Debug build ACN_RT_DEBUG2 (weights <- per-sample container sigma): which samples' field outputs differ
between runs, and where they sat (chunk-local sample index)."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "tests"))
import numpy as np
import torch
from test_batch_independence import _setup, _render

S = 64
for tag in ("k4", "k8"):
    d, specs, routing, bg = _setup(tag, "w:", None)
    rays = torch.from_numpy(np.ascontiguousarray(d["render:rays"])).cuda()
    runs = []
    with torch.no_grad():
        for _ in range(8):
            runs.append(_render(rays, None, specs, routing, bg, 0.0, S)[2].cpu().numpy())
    st = np.stack(runs)                       # (runs, N, S) sigma
    var = ~np.all(st == st[0:1], axis=0)      # samples whose sigma differs in some run
    idx = np.argwhere(var)
    print(tag, "samples with varying sigma", int(var.sum()), "of", var.size, flush=True)
    for ray, i in idx[:20]:
        vals = st[:, ray, i]
        loc = (ray % (1024 // S)) * S + i
        print(tag, "ray", int(ray), "sample", int(i), "chunk-local", int(loc), "distinct values", np.unique(vals).tolist(), flush=True)
