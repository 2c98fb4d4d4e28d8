"""Micro-benchmark of acn_hashgrid_bwd on ray-major samples (the training layout): 2000 rays x 96
samples in the unit cube, L=16, T=2^20.  Run once per library variant (ACNERF_LIB=...)."""
import os
import sys
import time

import torch

sys.path.insert(0, os.getcwd())
from adaptive_city_nerf_amd import ops  # noqa: E402
from oracle import oracle as O  # noqa: E402

dev = "cuda"
g = torch.Generator(device=dev).manual_seed(0)
R, S = 2000, 96
o = torch.rand(R, 3, device=dev, generator=g) * 0.2 + 0.05
d = torch.nn.functional.normalize(torch.rand(R, 3, device=dev, generator=g) + 0.2, dim=-1)
t = torch.linspace(0.0, 0.7, S, device=dev)
x = (o[:, None, :] + d[:, None, :] * t[None, :, None]).clamp(1e-6, 1 - 1e-6).reshape(-1, 3).contiguous()
gout = torch.randn(x.shape[0], 32, device=dev, generator=g)
res = O.level_resolutions(16, 16, 4096).tolist()
for _ in range(3):
    gt = ops.hashgrid_bwd(x, gout, res, 20, 2, 1)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(20):
    gt = ops.hashgrid_bwd(x, gout, res, 20, 2, 1)
torch.cuda.synchronize()
dt = (time.perf_counter() - t0) / 20 * 1e3
ref = O.hashgrid_bwd(x.cpu().numpy(), gout.cpu().numpy(), res, 16, 20, 2, 1)
err = float((gt.cpu() - torch.from_numpy(ref)).abs().max())
print(f"{os.environ.get('ACNERF_LIB', 'default')}: {dt:.3f} ms per call (incl. zero-fill), M={x.shape[0]}, "
      f"max|err| vs oracle {err:.2e}")
