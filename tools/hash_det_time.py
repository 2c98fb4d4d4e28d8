"""Time the hash-grid backward, float-atomic vs deterministic (sort + ordered sums), on a C5-shaped
batch: 1000 rays x 96 samples in one expert's unit box, the reference grid (L=16, 2^20, 16..4096)."""
import sys
from pathlib import Path

import torch

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO))
from adaptive_city_nerf_amd import ops  # noqa: E402
from oracle import oracle as O  # noqa: E402

g = torch.Generator().manual_seed(3)
o = torch.rand(1000, 1, 3, generator=g) * 0.6 + 0.2
d = torch.nn.functional.normalize(torch.randn(1000, 1, 3, generator=g), dim=-1) * 0.3
t = torch.linspace(0, 1, 96).view(1, -1, 1)
x = (o + d * t).reshape(-1, 3).clamp(1e-6, 1 - 1e-6).contiguous().cuda()
gy = (torch.randn(x.shape[0], 32, generator=g) * 1e-3).cuda()
res = O.level_resolutions(16, 16, 4096).tolist()
for det in (False, True):
    for _ in range(3):
        ops.hashgrid_bwd(x, gy, res, 20, 2, 1, deterministic=det)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        ops.hashgrid_bwd(x, gy, res, 20, 2, 1, deterministic=det)
    e1.record()
    torch.cuda.synchronize()
    print(f"{'deterministic' if det else 'atomic':14s} {e0.elapsed_time(e1) / 20:.4f} ms per call "
          f"(includes the 128 MiB gradient-table allocation + zeroing), {x.shape[0]} points", flush=True)
