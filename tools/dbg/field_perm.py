"""Is the fused field's per-point result independent of the other points of its wave-tile?  acn_field_fwd over
the K=8 fixture points in the given order and permuted (bitwise per point)."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "tests"))
import numpy as np
import torch
import goldens as G
from test_batch_independence import _setup
from adaptive_city_nerf_amd import ops

for tag in ("k4", "k8"):
    d, specs, routing, bg = _setup(tag, "w:", None)
    x = torch.from_numpy(np.ascontiguousarray(d["field:x_d"])).cuda()
    n = x.shape[0]
    g = torch.Generator(device="cuda").manual_seed(3)
    perm = torch.randperm(n, device="cuda", generator=g)
    for am in (None, 0):
        sp = specs if am is None else [specs[0]]
        a = ops.field_fwd(x, sp, routing, active_module=am)
        b = ops.field_fwd(x[perm].contiguous(), sp, routing, active_module=am)
        c = ops.field_fwd(x, sp, routing, active_module=am)
        bad = ~torch.all(a[perm] == b, dim=1)
        bad2 = ~torch.all(a == c, dim=1)
        print(tag, "active", am, "points", n, "perm differing", int(bad.sum()), "rerun differing", int(bad2.sum()),
              "max", float((a[perm] - b).abs().max()), flush=True)
