"""For rays whose routed render differs between two runs: the first sample whose weight differs, and how
many experts the oracle's routing gives that sample."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "tests"))
import numpy as np
import torch
import goldens as G
from oracle import oracle as O
from test_batch_independence import _setup, _render

S = 64
for tag in ("k4", "k8"):
    d, specs, routing, bg = _setup(tag, "w:", None)
    rays_np = np.ascontiguousarray(d["render:rays"])
    rays = torch.from_numpy(rays_np).cuda()
    sc = G.scene()["masks"][G.MASK[tag]]
    runs = []
    with torch.no_grad():
        for _ in range(6):
            runs.append([x.cpu().numpy() for x in _render(rays, None, specs, routing, bg, 0.0, S)])
    i = np.arange(S)
    step = np.float32(1.0) / np.float32(S - 1)
    u = np.where(i < S // 2, (step * i.astype(np.float32)).astype(np.float32),
                 (np.float32(1.0) - step * (S - 1 - i).astype(np.float32)).astype(np.float32)).astype(np.float32)
    t = (rays_np[:, 6:7] * (np.float32(1) - u) + rays_np[:, 7:8] * u).astype(np.float32)
    pts = (rays_np[:, None, :3] + rays_np[:, None, 3:6] * t[..., None]).astype(np.float32)
    W, _ = O.routing(pts.reshape(-1, 3), np.array(sc["centroids"], np.float32), sc["cluster_2d"], float(d["bm"]))
    nexp = (W.reshape(rays_np.shape[0], S, -1) > 0).sum(-1)
    for r in range(1, len(runs)):
        w0, w1 = runs[0][2], runs[r][2]
        bad = np.nonzero(~np.all(w0 == w1, axis=1))[0]
        for ray in bad[:6]:
            first = int(np.nonzero(w0[ray] != w1[ray])[0][0])
            print(tag, "run", r, "ray", int(ray), "first differing sample", first, "experts there", int(nexp[ray, first]),
                  "ray's multi-expert samples", np.nonzero(nexp[ray] > 1)[0].tolist()[:8],
                  "ray local in chunk", int(ray) % (1024 // S), flush=True)
