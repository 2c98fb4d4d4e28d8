"""Count samples whose routed-render field output (ACN_RT_DEBUG2 builds: weights <- sigma) varies over 8 runs."""
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
    with torch.no_grad():
        st = np.stack([_render(rays, None, specs, routing, bg, 0.0, S)[2].cpu().numpy() for _ in range(10)])
    var = ~np.all(st == st[0:1], axis=0)
    print(os.environ.get("VARIANT"), tag, "samples with varying output", int(var.sum()), "of", var.size, flush=True)
