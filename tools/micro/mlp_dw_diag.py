"""Phase cycles of mlp_bwd_dw_kernel (diagnostic build -DACN_DW_DIAG=1, ACNERF_LIB): per wave, shader-clock
cycles in tile_forward / output-gradient loads / stage rounds (barriers + LDS writes) / dW contraction /
dX chain / last layer + dh0 / flush, averaged over waves, at the meta-training size (M = 362,666)."""
import ctypes as C
import sys
import numpy as np
import torch

sys.path.insert(0, ".")
from adaptive_city_nerf_amd import _lib, ops  # noqa: E402

M = 362_666
g = torch.Generator(device="cuda").manual_seed(0)
ws = [((torch.rand(s, device="cuda", generator=g) - 0.5) * 0.4).contiguous() for s in ops.MLP_DW_SHAPES]
h0 = torch.rand(M, 32, device="cuda", generator=g) - 0.5
sh = torch.rand(M, 16, device="cuda", generator=g) - 0.5
gout = torch.randn(M, 4, device="cuda", generator=g) * 1e-6
out, _ = ops.mlp_train_fwd(h0, sh, ws, save=False)
for _ in range(3):
    ops.mlp_train_bwd_dw(h0, sh, out, gout, ws, want_h0=True)
torch.cuda.synchronize()
a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
a.record()
ops.mlp_train_bwd_dw(h0, sh, out, gout, ws, want_h0=True)
b.record()
torch.cuda.synchronize()
nblk = 256
buf = (C.c_ulonglong * (nblk * 4 * 8))()
L = _lib.lib()
fn = getattr(L, "acn_mlp_dw_diag", None)
print(f"call {a.elapsed_time(b) * 1e3:.1f} us")
if fn is None:
    sys.exit("not a diagnostic build")
fn.argtypes = [C.c_void_p, C.c_int]
assert fn(buf, nblk) == 0
d = np.frombuffer(buf, dtype=np.uint64).reshape(nblk * 4, 8).astype(np.float64)
names = ["tile_forward", "stage (barriers + LDS writes)", "dW contraction", "dX chain + relu", "grad loads",
         "last layer dX + dh0 store", "flush", "-"]   # counter index -> phase (mlp_train.hip DW_LAP)
order = [0, 4, 1, 2, 3, 5, 6]
tot = d[:, order].sum(1)
print(f"total shader cycles per wave: mean {tot.mean():.0f} (min {tot.min():.0f}, max {tot.max():.0f}) "
      f"= {tot.mean() / 2400:.1f} us at 2.4 GHz")
for i in order:
    print(f"  {names[i]:32s} {d[:, i].mean():10.0f}  {100 * d[:, i].mean() / tot.mean():5.1f}%")
