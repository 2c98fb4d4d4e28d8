"""Time the training MLP kernels (developer tool): fused backward (acn_mlp_train_bwd_dw) vs the split
path (saving forward + acn_mlp_train_bwd + batched GEMMs) at the meta-training (384k) and C5 (96k) sizes."""
import sys
import torch

sys.path.insert(0, ".")
from adaptive_city_nerf_amd import ops  # noqa: E402


def timeit(fn, n=20):
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
for M in (384_000, 96_000):
    h0 = torch.rand(M, 32, device="cuda", generator=g) - 0.5
    sh = torch.rand(M, 16, device="cuda", generator=g) - 0.5
    gout = torch.randn(M, 4, device="cuda", generator=g)
    out, save = ops.mlp_train_fwd(h0, sh, ws, save=True)
    t_fwd_save = timeit(lambda: ops.mlp_train_fwd(h0, sh, ws, save=True))
    t_fwd = timeit(lambda: ops.mlp_train_fwd(h0, sh, ws, save=False))
    t_dw = timeit(lambda: ops.mlp_train_bwd_dw(h0, sh, out, gout, ws, want_h0=True))
    t_dw_noh = timeit(lambda: ops.mlp_train_bwd_dw(h0, sh, out, gout, ws, want_h0=False))
    t_bwd = timeit(lambda: ops.mlp_train_bwd(save, out, gout, ws, want_h0=True))
    print(f"M={M}: fwd(save) {t_fwd_save:.1f} us, fwd {t_fwd:.1f} us, bwd_dw {t_dw:.1f} us "
          f"(no dh0 {t_dw_noh:.1f}), split bwd kernel {t_bwd:.1f} us (+ GEMMs)", flush=True)
