"""Which role bounds the producer / consumer MLP backward (developer tool): acn_mlp_train_bwd_dw at
the meta batch (362,666 samples, the meta step's average launch) for the default fp16x3 and the use_amp kernels,
on whatever libacnerf.so ACNERF_LIB names -- the regular build, or the diagnostic builds without the
weight-gradient contraction (ACN_DIAG_NODW: the producers' time) or without the producers' forward recompute and
dX chain (ACN_DIAG_NOPROD: the consumers' time)."""
import sys
import torch

sys.path.insert(0, ".")
from adaptive_city_nerf_amd import ops  # noqa: E402


def timeit(fn, n=30):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(n):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / n * 1e3


g = torch.Generator(device="cuda").manual_seed(0)
ws = [((torch.rand(s, device="cuda", generator=g) - 0.5) * 0.4).contiguous() for s in ops.MLP_DW_SHAPES]
M = 362_666
h0 = torch.rand(M, 32, device="cuda", generator=g) - 0.5
sh = torch.rand(M, 16, device="cuda", generator=g) - 0.5
gout = torch.randn(M, 4, device="cuda", generator=g) * 1e-4
tag = sys.argv[1] if len(sys.argv) > 1 else "?"
for prec in ("fp16x3", "amp"):
    out, _ = ops.mlp_train_fwd(h0, sh, ws, save=False, precision=prec)
    t = timeit(lambda: ops.mlp_train_bwd_dw(h0, sh, out, gout * (65536.0 if prec == "amp" else 1.0), ws,
                                            want_h0=False, precision=prec))
    print(f"{tag} {prec}: bwd_dw {t:.1f} us", flush=True)
