"""ACN_RT_CHECK builds: per ray, OR of self-check flags (1: a second load of the ray differs, 2: a second
evaluation of the same sample's field differs)."""
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
    tot = np.zeros(4, int)
    with torch.no_grad():
        for _ in range(10):
            dep = _render(rays, None, specs, routing, bg, 0.0, S)[1].cpu().numpy().astype(int)
            for b in range(3):
                tot[b] += int(((dep >> b) & 1).sum())
    print(tag, "rays flagged: ray reload mismatch", tot[0], "field re-evaluation mismatch", tot[1], flush=True)
