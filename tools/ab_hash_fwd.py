"""Hash-grid forward A/B at the meta-training batch (developer tool).

python tools/ab_hash_fwd.py [--points 384000] [--log2T 19] [--steps 50]

Times acn_hashgrid_fwd (the standalone HashGridEncoder forward the meta step and the adapt steps call) on
points along random rays through the unit cube (96 consecutive samples per ray, as a task's support batch lays
them out), L = 16, F = 2, resolutions 16 .. 4096 (the reference grid), Linear and Smoothstep, and prints one
JSON line per interpolation with the HIP-event time per launch, the algorithmic table bytes (8 corners x 8 B
per point and level) and an output checksum (compare it across ACNERF_LIB builds: the gather forms must agree
bit for bit)."""
import argparse
import json
import math
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--points", type=int, default=384000)
    ap.add_argument("--log2T", type=int, default=19)
    ap.add_argument("--steps", type=int, default=50)
    a = ap.parse_args()
    from adaptive_city_nerf_amd import ops
    dev = torch.device("cuda", 0)
    g = torch.Generator(device="cpu").manual_seed(0)
    S = 96
    n = (a.points + S - 1) // S
    o = torch.rand(n, 3, generator=g)
    d = torch.nn.functional.normalize(torch.randn(n, 3, generator=g), dim=1)
    t = torch.linspace(0.0, 0.8, S)
    x = (o[:, None, :] * 0.5 + 0.25 + d[:, None, :] * t[None, :, None]).clamp(0.0, 1.0).reshape(-1, 3)[: a.points]
    x = x.contiguous().to(dev)
    L, F = 16, 2
    b = math.exp((math.log(4096) - math.log(16)) / (L - 1))
    res = [int(math.floor(16 * b ** l)) for l in range(L)]
    table = (torch.rand((L << a.log2T, F), generator=g) * 2e-3 - 1e-3).to(dev)
    for interp, name in ((1, "Linear"), (2, "Smoothstep")):
        for _ in range(5):
            y = ops.hashgrid_fwd(x, table, res, a.log2T, F, interp)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.steps):
            y = ops.hashgrid_fwd(x, table, res, a.log2T, F, interp)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / a.steps
        alg = a.points * L * 8 * 8
        print(json.dumps({"interp": name, "points": a.points, "log2T": a.log2T, "us_per_launch": round(ms * 1e3, 2),
                          "table_bytes_algorithmic": alg, "achieved_GBps": round(alg / (ms * 1e-3) / 1e9, 1),
                          "checksum": float(y.double().sum()), "abs_checksum": float(y.double().abs().sum())}),
              flush=True)


if __name__ == "__main__":
    main()
