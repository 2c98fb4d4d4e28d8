"""Fast-weight module surface (reference: models/metamodule/metamodule.py:13-192).

MAML/FOMAML inject adapted MLP weights through an OrderedDict ``params`` keyed like
``submodules.0.sigma_trunk.0.linear.weight`` (pipelines/offline_stage/meta_core.py:26-66).  The
HIP field/render kernels read those tensors' device pointers directly, so the same dicts drive
the fused path; this module keeps the resolution rules (get_subdict prefix stripping,
per-layer fallback to the module's own parameters) identical.
"""
from __future__ import annotations

import re
import warnings
from collections import OrderedDict
from typing import Dict, Optional

import torch
import torch.nn as nn

from .trunc_exp import trunc_exp


class MetaModule(nn.Module):
    """Module whose parameters may be overridden per call by a ``params`` dict."""

    def __init__(self):
        super().__init__()
        self._children_modules_parameters_cache = dict()

    def meta_named_parameters(self, prefix: str = "", recurse: bool = True):
        gen = self._named_members(
            lambda module: module._parameters.items() if isinstance(module, MetaModule) else [],
            prefix=prefix, recurse=recurse)
        for elem in gen:
            yield elem

    def meta_parameters(self, recurse: bool = True):
        for _, p in self.meta_named_parameters(recurse=recurse):
            yield p

    def get_subdict(self, params: Optional[Dict[str, torch.Tensor]], key: Optional[str] = None):
        """Entries of ``params`` under ``key.`` with the prefix removed (None if absent)."""
        if params is None:
            return None
        all_names = tuple(params.keys())
        ck = (key, all_names)
        if ck not in self._children_modules_parameters_cache:
            if key is None:
                self._children_modules_parameters_cache[ck] = all_names
            else:
                rx = re.compile(rf"^{re.escape(key)}\.(.+)")
                self._children_modules_parameters_cache[ck] = [rx.sub(r"\1", k) for k in all_names if rx.match(k)]
        names = self._children_modules_parameters_cache[ck]
        if not names:
            warnings.warn(f"Module `{self.__class__.__name__}` has no parameter for submodule `{key}` in "
                          f"`params`.\nUsing default parameters. Provided keys: [{', '.join(all_names)}]",
                          stacklevel=2)
            return None
        return OrderedDict((n, params[f"{key}.{n}"]) for n in names)


class MetaSequential(nn.Sequential, MetaModule):
    def forward(self, input, params: Optional[Dict[str, torch.Tensor]] = None):
        for name, module in self._modules.items():
            if isinstance(module, MetaModule):
                input = module(input, params=self.get_subdict(params, name))
            elif isinstance(module, nn.Module):
                input = module(input)
            else:
                raise TypeError(f"The module must be a `nn.Module` or `MetaModule`. Got: {type(module)}")
        return input


_SPLITK_ROWS = 2048     # rows per split-K slice of the weight-gradient GEMM
_SPLITK_MIN_ROWS = 16384


def _wgrad_splitk(g: torch.Tensor, x: torch.Tensor) -> torch.Tensor:
    """g^T @ x for tall (M x out), (M x in) operands as a batched GEMM over M-slices + a sum.
    The field's weight gradients contract over M = rays x samples (~1e5) with out, in <= 64: as
    one GEMM that is a 2-tile problem (rocBLAS ran it at ~3 TFLOP/s, 0.2-0.3 ms per layer); split
    over M it fills the GPU."""
    M = g.shape[0]
    main = (M // _SPLITK_ROWS) * _SPLITK_ROWS
    gw = torch.bmm(g[:main].view(-1, _SPLITK_ROWS, g.shape[1]).transpose(1, 2),
                   x[:main].view(-1, _SPLITK_ROWS, x.shape[1])).sum(0)
    if main < M:
        gw = gw + g[main:].t() @ x[main:]
    return gw


def _bias_grad(g: torch.Tensor) -> torch.Tensor:
    """Column sums of the tall (M x out) output gradient.  torch's dim-0 reduction is fast for 64
    columns but 5-15x slower for the 15-, 3- and 1-wide heads (490 us vs 37 us at M = 384k, measured
    with tools/micro/bias_sum.py); reducing 2048-row slices first is uniform across widths."""
    M, C = g.shape
    if M < _SPLITK_MIN_ROWS or C % 64 == 0:
        return g.sum(0)
    main = (M // _SPLITK_ROWS) * _SPLITK_ROWS
    gb = g[:main].view(-1, _SPLITK_ROWS, C).sum(1).sum(0)
    return gb + g[main:].sum(0) if main < M else gb


class _LinearFn(torch.autograd.Function):
    """y = x W^T + b (one addmm) with a split-K weight gradient; the backward is written with
    differentiable ops, so second-order MAML (create_graph=True) still works through it."""

    @staticmethod
    def forward(ctx, x, w, b):
        ctx.save_for_backward(x, w)
        ctx.has_bias = b is not None
        return torch.addmm(b, x, w.t()) if b is not None else x @ w.t()

    @staticmethod
    def backward(ctx, g):
        x, w = ctx.saved_tensors
        gx = g @ w if ctx.needs_input_grad[0] else None
        gw = _wgrad_splitk(g, x) if ctx.needs_input_grad[1] else None
        gb = _bias_grad(g) if ctx.has_bias and ctx.needs_input_grad[2] else None
        return gx, gw, gb


class MetaLinear(nn.Linear, MetaModule):
    """y = x @ W^T + b with optional fast weights {'weight', 'bias'} (metamodule.py:129-156)."""

    def forward(self, inputs: torch.Tensor, params: Optional[Dict[str, torch.Tensor]] = None):
        if params is None:
            weight, bias = self.weight, self.bias
        else:
            weight = params.get("weight", self.weight)
            bias = params.get("bias", self.bias)
        if inputs.dtype != weight.dtype:
            inputs = inputs.to(weight.dtype)
        lead = inputs.shape[:-1]
        flat = inputs.reshape(-1, inputs.shape[-1])
        if flat.is_cuda and flat.shape[0] >= _SPLITK_MIN_ROWS and torch.is_grad_enabled():
            return _LinearFn.apply(flat, weight, bias).view(*lead, weight.shape[0])
        out = inputs.matmul(weight.t())
        if bias is not None:
            out = out + bias
        return out


class MetaBatchLinear(nn.Linear, MetaModule):
    """Batched fast-weight linear: inputs (B,N,in), weight (B,out,in), bias (B,out)."""

    def forward(self, inputs: torch.Tensor, params: Optional[Dict[str, torch.Tensor]] = None):
        if params is None:
            params = OrderedDict(self.named_parameters())
            for name, p in params.items():
                params[name] = p[None, ...].repeat((inputs.size(0),) + (1,) * len(p.shape))
        weight = params["weight"]
        bias = params.get("bias", None)
        if weight.dim() == 2:
            weight = weight.unsqueeze(0)
        if bias is not None:
            if bias.dim() == 1:
                bias = bias.unsqueeze(0)
            elif bias.dim() == 3 and bias.shape[1] == 1:
                bias = bias.squeeze(1)
        out = torch.bmm(weight, inputs.transpose(1, 2)).transpose(1, 2)
        if bias is not None:
            out = out + bias.unsqueeze(1)
        return out


class MetaLayerBlock(MetaModule):
    """Linear + activation (relu / sigmoid / softplus / trunc_exp / identity)."""

    def __init__(self, dim_in: int, dim_out: int, activation: Optional[str] = None, batched: bool = False):
        super().__init__()
        self.linear = MetaBatchLinear(dim_in, dim_out) if batched else MetaLinear(dim_in, dim_out)
        if activation is None:
            self.act = nn.Identity()
        elif activation.lower() == "relu":
            self.act = nn.ReLU()
        elif activation.lower() == "sigmoid":
            self.act = nn.Sigmoid()
        elif activation.lower() == "softplus":
            self.act = nn.Softplus()
        elif activation.lower() == "trunc_exp":
            self.act = trunc_exp
        else:
            raise ValueError(f"Unsupported activation: {activation}")

    def forward(self, x: torch.Tensor, params: Optional[OrderedDict] = None):
        return self.act(self.linear(x, params=self.get_subdict(params, "linear")))
