"""Encoders of the hot path on MI355X (reference interface: models/encodings.py).

HashGridEncoder and SHEncoder keep the reference's constructor arguments, attributes, parameter
names (``hash_table``, state-dict compatible) and forward semantics -- the numerics are those of
the reference's pure-Torch fallback (what the reference runs on ROCm, where tinycudann is
absent), reproduced bit-exactly by the HIP kernels (tests/test_gpu_kernels.py).  Every value of
``implementation`` ("tcnn", "torch", "hip") runs the HIP kernels; there is no CPU path.
"""
from __future__ import annotations

import contextlib
import math
import threading
from typing import Literal, Optional

import torch
import torch.nn as nn

from . import ops
from ._lib import INTERP, AcnError

MAX_SH_DEGREE = 4
INTERPOLATIONS = ["Nearest", "Linear", "Smoothstep"]


def num_sh_bases(degree: int) -> int:
    assert degree <= MAX_SH_DEGREE, f"We don't support degree > {MAX_SH_DEGREE}."
    return (degree + 1) ** 2


def components_from_spherical_harmonics(degree: int, directions: torch.Tensor) -> torch.Tensor:
    """Real SH components of UNIT directions (encodings.py:27-81).  Elementwise utility kept for
    API compatibility; the encoders below use the fused HIP kernel (which also normalises)."""
    assert 0 <= degree <= MAX_SH_DEGREE
    assert directions.shape[-1] == 3
    x, y, z = directions[..., 0], directions[..., 1], directions[..., 2]
    xx, yy, zz = x * x, y * y, z * z
    c = directions.new_zeros((*directions.shape[:-1], num_sh_bases(degree)))
    c[..., 0] = 0.28209479177387814
    if degree > 0:
        c[..., 1] = 0.4886025119029199 * y
        c[..., 2] = 0.4886025119029199 * z
        c[..., 3] = 0.4886025119029199 * x
    if degree > 1:
        c[..., 4] = 1.0925484305920792 * x * y
        c[..., 5] = 1.0925484305920792 * y * z
        c[..., 6] = 0.9461746957575601 * zz - 0.31539156525251999
        c[..., 7] = 1.0925484305920792 * x * z
        c[..., 8] = 0.5462742152960396 * (xx - yy)
    if degree > 2:
        c[..., 9] = 0.5900435899266435 * y * (3 * xx - yy)
        c[..., 10] = 2.890611442640554 * x * y * z
        c[..., 11] = 0.4570457994644658 * y * (5 * zz - 1)
        c[..., 12] = 0.3731763325901154 * z * (5 * zz - 3)
        c[..., 13] = 0.4570457994644658 * x * (5 * zz - 1)
        c[..., 14] = 1.445305721320277 * z * (xx - yy)
        c[..., 15] = 0.5900435899266435 * x * (xx - 3 * yy)
    if degree > 3:
        c[..., 16] = 2.5033429417967046 * x * y * (xx - yy)
        c[..., 17] = 1.7701307697799304 * y * z * (3 * xx - yy)
        c[..., 18] = 0.9461746957575601 * x * y * (7 * zz - 1)
        c[..., 19] = 0.6690465435572892 * y * z * (7 * zz - 3)
        c[..., 20] = 0.10578554691520431 * (35 * zz * zz - 30 * zz + 3)
        c[..., 21] = 0.6690465435572892 * x * z * (7 * zz - 3)
        c[..., 22] = 0.47308734787878004 * (xx - yy) * (7 * zz - 1)
        c[..., 23] = 1.7701307697799304 * x * z * (xx - 3 * yy)
        c[..., 24] = 0.6258357354491761 * (xx * (xx - 3 * yy) - yy * (3 * xx - yy))
    return c


class SHEncoder(nn.Module):
    """Real spherical harmonics of degree levels-1 (encodings.py:84-151) on the HIP kernel."""

    def __init__(self, levels: int = 4, implementation: Literal["tcnn", "torch", "hip"] = "tcnn") -> None:
        super().__init__()
        if levels <= 0 or levels > MAX_SH_DEGREE + 1:
            raise ValueError(f"Supported levels ∈ [1, {MAX_SH_DEGREE + 1}], got {levels}")
        self.levels = int(levels)
        self.degree = self.levels - 1
        self._out_dim = self.levels ** 2
        self.implementation = "hip"

    @property
    def out_dim(self) -> int:
        return self._out_dim

    def forward(self, d: torch.Tensor) -> torch.Tensor:
        assert d.shape[-1] == 3, f"Expected (...,3); got {tuple(d.shape)}"
        if d.requires_grad:
            raise AcnError("SHEncoder: gradients w.r.t. directions are not implemented on the HIP path")
        return ops.sh_fwd(d, self.levels).to(d.dtype)


_ACC = threading.local()


@contextlib.contextmanager
def accumulate_table_grad():
    """Inside this context a hash-grid backward scatters the table gradient straight into the table's
    existing ``.grad`` buffer (float atomics onto the accumulated values) and hands autograd None for the
    table: no 128 MiB zero-fill for a fresh gradient and no 128 MiB AccumulateGrad add per backward.
    The sum is the same (up to fp32 summation order, which the atomics leave unordered anyway).  Used by
    the graph-replayed meta step, whose persistent .grad buffers are accumulated over its tasks."""
    prev = getattr(_ACC, "on", False)
    _ACC.on = True
    try:
        yield
    finally:
        _ACC.on = prev


class _HashGridFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x01, table, enc):
        ctx.save_for_backward(x01)
        ctx.enc = enc
        ctx.table = table
        return ops.hashgrid_fwd(x01, table, enc._res_host, enc.log2_hashmap_size, enc.features_per_level,
                                enc._interp_code)

    @staticmethod
    def backward(ctx, g):
        (x01,) = ctx.saved_tensors
        enc = ctx.enc
        if ctx.needs_input_grad[0]:
            raise AcnError("HashGridEncoder: gradients w.r.t. the input points are not implemented on the HIP "
                           "path (the reference pipelines never request them)")
        gt = None
        if ctx.needs_input_grad[1]:
            tab = ctx.table
            into = tab.grad if getattr(_ACC, "on", False) and not torch.are_deterministic_algorithms_enabled() else None
            if into is not None and into.shape == tab.shape and into.dtype == torch.float32 and into.is_contiguous():
                ops.hashgrid_bwd(x01, g.contiguous(), enc._res_host, enc.log2_hashmap_size, enc.features_per_level,
                                 enc._interp_code, out=into)
                return None, None, None
            gt = ops.hashgrid_bwd(x01, g.contiguous(), enc._res_host, enc.log2_hashmap_size, enc.features_per_level,
                                  enc._interp_code)
        return None, gt, None


class HashGridEncoder(nn.Module):
    """Instant-NGP multiresolution hash grid (encodings.py:158-381) on the HIP kernels.

    forward(x: (...,3) in [0,1]) -> (..., levels * features_per_level), level-major.  The table
    is the fp32 parameter ``hash_table`` of shape (levels * 2**log2_hashmap_size, F), initialised
    U(-hash_init_scale, hash_init_scale) as in the reference (:264-268).
    """

    def __init__(self, levels: int = 16, min_res: int = 16, max_res: int = 4096, log2_hashmap_size: int = 19,
                 features_per_level: int = 2, hash_init_scale: float = 1e-3,
                 implementation: Literal["tcnn", "torch", "hip"] = "tcnn",
                 interpolation: Optional[Literal["Nearest", "Linear", "Smoothstep"]] = None) -> None:
        super().__init__()
        self.levels = int(levels)
        self.min_res = int(min_res)
        self.max_res = int(max_res)
        self.features_per_level = int(features_per_level)
        self.log2_hashmap_size = int(log2_hashmap_size)
        self.hash_init_scale = float(hash_init_scale)
        self.hash_table_size = 2 ** self.log2_hashmap_size
        self.interpolation = interpolation
        L = self.levels
        self.growth_factor = 1.0 if L <= 1 else float(math.exp((math.log(self.max_res) - math.log(self.min_res)) / (L - 1)))
        lv = torch.arange(L, dtype=torch.float32)
        scalings = torch.floor(self.min_res * (self.growth_factor ** lv)).to(torch.int32)   # float32 pow, as :211-215
        self.register_buffer("level_resolutions", scalings, persistent=False)
        self.register_buffer("level_offsets", torch.arange(L, dtype=torch.int64) * self.hash_table_size,
                             persistent=False)
        self._res_host = [int(v) for v in scalings.tolist()]
        self._out_dim = self.levels * self.features_per_level
        self.implementation = "hip"
        T = self.hash_table_size * self.levels
        F = self.features_per_level
        self.hash_table = nn.Parameter((torch.rand(T, F) * 2 - 1) * self.hash_init_scale)
        self.register_buffer("hash_primes", torch.tensor([1, 2654435761, 805459861], dtype=torch.int64),
                             persistent=False)
        if self.interpolation is not None and self.interpolation not in INTERPOLATIONS:
            self.interpolation = "Linear"
        self._interp_code = INTERP[self.interpolation or "Linear"]

    @property
    def out_dim(self) -> int:
        return self._out_dim

    def get_out_dim(self) -> int:
        return self._out_dim

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        assert x.shape[-1] == 3, f"Expected (...,3), got {tuple(x.shape)}"
        y = _HashGridFn.apply(x, self.hash_table, self)
        return y.to(x.dtype) if x.dtype != torch.float32 else y


class FrequencyEncoder(nn.Module):
    """NeRF positional encoding (encodings.py:387-444); not on the default hot path
    (dir_encoding='spherical').  Elementwise torch ops, kept for interface completeness."""

    def __init__(self, in_dim: int, pe_dim: int, include_input: bool = True, use_pi: bool = False):
        super().__init__()
        self.in_dim = int(in_dim)
        self.pe_dim = int(pe_dim)
        self.include_input = bool(include_input)
        self.use_pi = bool(use_pi)
        self.register_buffer("bands", 2.0 ** torch.arange(self.pe_dim, dtype=torch.float32), persistent=False)

    @property
    def out_dim(self) -> int:
        return self.in_dim * (2 * self.pe_dim + (1 if self.include_input else 0))

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        assert x.shape[-1] == self.in_dim, f"Expected (...,{self.in_dim}), got {tuple(x.shape)}"
        fb = self.bands.to(dtype=x.dtype, device=x.device)
        xin = x * (x.new_tensor(math.pi) if self.use_pi else 1)
        xe = xin[..., None] * fb
        pe = torch.cat([torch.cos(xe), torch.sin(xe)], dim=-1).reshape(*x.shape[:-1], -1)
        return torch.cat([x, pe], dim=-1) if self.include_input else pe

    torch_forward = forward
