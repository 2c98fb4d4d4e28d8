"""Section timings of composite_mse_train_kernel (the fused C5 compositing glue) from its ACN_CM_PROF=1 build
(tools/build_variants.sh cmprof:render.hip:"-DACN_CM_PROF=1"; run with ACNERF_LIB=build_variants/libacnerf_cmprof.so).
Lane 0 of every ray's wave stamps wall_clock64() at: 0 ray start, 1 after the blend + t staging, 2 after the
background head (+ LDS sync), 3 after forward compositing + loss gradient, 4 after the two backward sweeps,
5 after the blend backward.  Prints per-section medians over the rays of the train_k8 fixture batches."""
import ctypes
import os
import sys
from types import SimpleNamespace

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "tests"))
import numpy as np
import torch

import goldens as G
from test_train import P
from test_module_api import build_model, reference_state_dict
from adaptive_city_nerf_amd import _lib
from adaptive_city_nerf_amd import optim as O
from adaptive_city_nerf_amd import routed_train as RT

L = _lib.lib()
fetch = L.acn_debug_cmprof_fetch
fetch.argtypes, fetch.restype = [ctypes.c_void_p, ctypes.c_int], ctypes.c_int
fetchb = L.acn_debug_cmblk_fetch
fetchb.argtypes, fetchb.restype = [ctypes.c_void_p, ctypes.c_int], ctypes.c_int
bb = np.zeros((4096, 4), np.uint64)
d = G.load("train_k8")
Pk = SimpleNamespace(**{**vars(P), "ray_samples": 96, "chunk_points": 4_000_000})
m, _ = build_model("k8")
m.load_state_dict(reference_state_dict(d, 8, "w:"))
m = m.cuda().train()
opt = O.build_optimizer(Pk, m)
st = RT.RoutedAdaptStep(Pk, m, 1000, opt, grad_clip=1.0, graph=False, jitter="given")
buf = np.zeros((4096, 8), np.uint64)
names = ["blend+t", "bg+sync", "fwd+loss", "bwd sweeps", "blend bwd"]
for i in range(4):
    r, c, u = (torch.from_numpy(d[f"train{i % 3}:{k}"]).cuda() for k in ("rays", "rgbs", "u"))
    st(r, c, jitter_u=u)
    torch.cuda.synchronize()
    n = fetch(buf.ctypes.data, 1000)
    t = buf[:n].astype(np.float64)
    sec = np.diff(t[:, :6], axis=1) / 100.0   # wall_clock64 at 100 MHz -> us
    tot = (t[:, 5] - t[:, 0]) / 100.0
    span = (t[:, 5].max() - t[:, 0].min()) / 100.0
    print(f"step {i}: " + ", ".join(f"{nm} {np.median(sec[:, k]):.2f}" for k, nm in enumerate(names)) +
          f" | per-ray total median {np.median(tot):.2f} max {tot.max():.2f} | first start -> last end {span:.2f} us"
          f" | start spread {(t[:, 0].max() - t[:, 0].min()) / 100.0:.2f} us", flush=True)
    nb = fetchb(bb.ctypes.data, 250)
    q = bb[:nb].astype(np.float64)
    t0 = q[:, 0].min()
    lastb = int(np.argmax(q[:, 3]))
    print(f"   blocks: entry spread {(q[:, 0].max() - t0) / 100:.2f}, ray loops end (max) {(q[:, 1].max() - t0) / 100:.2f}, "
          f"padding end (max) {(q[:, 2].max() - t0) / 100:.2f}, last block {lastb} done {(q[lastb, 3] - t0) / 100:.2f} us "
          f"(its padding end {(q[lastb, 2] - t0) / 100:.2f}); rays: first start {(t[:, 0].min() - t0) / 100:.2f}", flush=True)
