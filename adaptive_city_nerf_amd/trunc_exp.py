"""trunc_exp: exp with a dtype-dependent clamp and the clamped-input backward.

Mirrors the reference's models/trunc_exp.py:22-61 interface (``trunc_exp(x)``); inside the fused
HIP field kernel the same clamp (+-88.722839111 for fp32) is applied on device (acn_device.h).
This autograd form is used by the differentiable (training) composition.
"""
import torch

_EXP_MAX = {
    torch.float16: 11.089866488,
    torch.bfloat16: 88.722839111,
    torch.float32: 88.722839111,
    torch.float64: 709.782712893,
}


def _clamp(x: torch.Tensor) -> torch.Tensor:
    m = _EXP_MAX.get(x.dtype, _EXP_MAX[torch.float32])
    return x.clamp(-m, m)


class TruncExp(torch.autograd.Function):
    """Forward exp(clamp(x)); backward g * exp(xc) with xc saved from the forward (models/trunc_exp.py:
    43-57).  Under create_graph the backward is differentiable in g only -- xc is a constant of the
    saved forward, exactly as in the reference, so second-order MAML matches it term for term."""

    @staticmethod
    def forward(ctx, x):
        xc = _clamp(x)
        ctx.save_for_backward(xc)
        return torch.exp(xc)

    @staticmethod
    def backward(ctx, g):
        (xc,) = ctx.saved_tensors
        return g * torch.exp(xc)


def trunc_exp(x: torch.Tensor) -> torch.Tensor:
    return TruncExp.apply(x)
