"""Latency of the training-loss launches at the meta step's size (developer tool).

python tools/micro/loss_micro.py

n = 4000 rays x 3 (the meta support batch).  Times, by HIP events over 200 back-to-back calls on cuda:0:
acn_mse_linear_fwd_ws (multi-workgroup, last-workgroup reduction), acn_mse_linear_fwd (one workgroup) and
acn_mse_linear_bwd, each alone and each after a 16 MiB device write (dirty L2 lines for the fences to write
back); the write alone is timed too and subtracted."""
from __future__ import annotations

import ctypes as C
import json
import sys
from pathlib import Path

import torch

REPO = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(REPO))


def time_ms(fn, reps: int = 200) -> float:
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3   # us


def main():
    from adaptive_city_nerf_amd import _lib, ops
    dev = torch.device("cuda", 0)
    L = _lib.lib()
    n = 12000
    g = torch.Generator(dev).manual_seed(1)
    pred = torch.rand(n, device=dev, generator=g)
    gt = torch.rand(n, device=dev, generator=g)
    loss = torch.empty((), device=dev)
    gl = torch.ones((), device=dev)
    gp = torch.empty(n, device=dev)
    ws = torch.zeros(int(L.acn_mse_linear_workspace_bytes()), dtype=torch.uint8, device=dev)
    big = torch.empty(4 << 20, device=dev)
    s = C.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    P = ops.ptr

    def fwd_ws():
        L.acn_mse_linear_fwd_ws(P(pred), P(gt), n, P(loss), P(ws), ws.numel(), s)

    def fwd_one():
        L.acn_mse_linear_fwd(P(pred), P(gt), n, P(loss), s)

    def bwd():
        L.acn_mse_linear_bwd(P(pred), P(gt), n, P(gl), P(gp), s)

    def dirty():
        big.fill_(1.0)

    res = {"n": n}
    t_dirty = time_ms(dirty)
    res["fill_16MiB_us"] = round(t_dirty, 2)
    for name, fn in (("fwd_ws", fwd_ws), ("fwd_one_wg", fwd_one), ("bwd", bwd)):
        res[name + "_us"] = round(time_ms(fn), 2)
        res[name + "_after_fill_us"] = round(time_ms(lambda fn=fn: (dirty(), fn())) - t_dirty, 2)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
