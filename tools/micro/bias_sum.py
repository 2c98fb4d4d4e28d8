"""Micro-benchmark: column sums of a tall (M, C) fp32 gradient (the MetaLinear bias gradient)."""
import time
import torch

dev = "cuda"
for M, Cc in ((384000, 64), (384000, 3), (192000, 64), (384000, 15)):
    g = torch.randn(M, Cc, device=dev)
    ones = torch.ones(M, device=dev)
    S = 2048
    main = (M // S) * S
    cands = {
        "sum0": lambda: g.sum(0),
        "ones@g": lambda: ones @ g,
        "g.t()@ones": lambda: g.t() @ ones,
        "bmm_slices": lambda: torch.bmm(torch.ones(main // S, 1, S, device=dev), g[:main].view(-1, S, Cc)).sum((0, 1))
        + g[main:].sum(0),
        "view_sum1_sum0": lambda: g[:main].view(-1, S, Cc).sum(1).sum(0) + g[main:].sum(0),
    }
    ref = g.double().sum(0)
    for name, fn in cands.items():
        for _ in range(3):
            y = fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(50):
            y = fn()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / 50 * 1e6
        err = float((y.double() - ref).abs().max())
        print(f"M={M} C={Cc} {name:16s} {dt:8.1f} us  maxerr={err:.2e}")
