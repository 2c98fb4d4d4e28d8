import os, sys, numpy as np, torch
sys.path.insert(0, '/root/repo'); sys.path.insert(0, '/root/repo/tests')
import goldens as G
from test_gpu_kernels import _spec, _t
from adaptive_city_nerf_amd import ops
d = G.load("render_k4"); mask = G.MASK["k4"]; sc = G.scene()["masks"][mask]; K = 4
for variant, prefix in (("render", "w:"), ("render_hi", "hiw:")):
    specs = [_spec(d, k, mask, prefix=prefix) for k in range(K)]
    routing = ops.make_routing(torch.tensor(sc["centroids"]), K, True, float(d["bm"]))
    bgw = {k[len("bg_mlp."):]: _t(v) for k, v in G.bg_weights(d, prefix).items()}
    bg, keep = ops.make_background("mlp", mlp=bgw)
    rays = _t(d["render:rays"])
    rgb, depth, w, acc = ops.render_stratified(rays, 64, specs, routing, None, bg)
    w = w.cpu().numpy(); ref = d[f"{variant}:weights"]
    err = np.abs(w - ref).max(1)
    bad = np.argsort(-err)[:8]
    print(variant, "max", err.max(), "rays over 1e-6:", (err > 1e-6).sum(), "worst", bad.tolist(), err[bad].tolist())
    # field check on the worst ray's samples: compare container field vs oracle expectations
    r = d["render:rays"][bad[0]]
    print("worst ray near/far", r[6:8])
