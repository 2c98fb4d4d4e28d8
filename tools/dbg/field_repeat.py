"""Run-to-run probe of acn_field_fwd (developer tool): the K = 4 fixture's field inputs evaluated
`reps` times through the container (soft routing) and one expert; per call, the samples that differ bitwise from
the first call and the worst sigma error against the reference fixture.  ACNERF_LIB selects the library."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "tests"))
import numpy as np
import torch

import goldens as G
from test_gpu_kernels import _spec, _sigma_close, _t
from adaptive_city_nerf_amd import ops

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 200
lib = os.path.basename(os.environ.get("ACNERF_LIB", "default"))
for tag in ("k4", "k8"):
    d = G.load(f"render_{tag}")
    mask = G.MASK[tag]
    sc = G.scene()["masks"][mask]
    K = len(sc["centroids"])
    specs = [_spec(d, k, mask) for k in range(K)]
    routing = ops.make_routing(torch.tensor(sc["centroids"]), K, True, float(d["bm"]))
    x = _t(d["field:x_d"])
    x = torch.cat([x] * 16)            # 16 copies: more waves in flight, more chances
    refc = np.concatenate([d["field:y_container"]] * 16)
    first = None
    bad_calls = bad_samples = 0
    worst = 0.0
    for it in range(reps):
        y = ops.field_fwd(x, specs, routing)
        if first is None:
            first = y.clone()
        diff = (y != first).any(dim=1)
        nd = int(diff.sum())
        if nd:
            bad_calls += 1
            bad_samples += nd
        worst = max(worst, float(_sigma_close(y[:, 3].cpu().numpy(), refc[:, 3])))
    print(f"{lib} {tag}: {reps} calls x {x.shape[0]} samples: {bad_calls} calls / {bad_samples} samples differ from "
          f"the first; worst sigma error vs reference {worst:.3g}", flush=True)
