"""Stratified volumetric rendering (reference interface: nerfs/ray_rendering.py:23-345, 564-627).

``render_rays`` / ``render_rays_stratified`` / ``render_image`` / ``volume_render`` keep the
reference's signatures and return values.  Without autograd (eval, rendering, viewer) a whole
``render_rays`` call is ONE fused HIP launch (acn_render_stratified_fwd): t-values -> points ->
routing -> every needed expert's hash grid + MLPs on fp32 MFMA -> soft blend -> background ->
front-to-back compositing; the (N,S,4) field output and the (N*S,6) point table the reference
materialises never exist.  With autograd (training) the call composes the differentiable
per-expert forward (HIP hash grid + fast-weight MetaLinear chain) with the reference's
compositing formulas.

Extensions (not in the reference): ``early_stop_tau`` (default 0 = off) stops a ray once its
transmittance drops below tau; the composite then differs from the reference by at most 2*tau.
``jitter_u`` (N, S) supplies the uniforms of the training-mode jitter (the reference draws them
with torch.rand_like, ray_rendering.py:286) so a training step can be reproduced exactly.
"""
from __future__ import annotations

import os
import threading
import warnings
from contextlib import contextmanager
from typing import Optional, Tuple

import torch
from torch import Tensor

from . import nerfacc, occ_ops, ops
from ._lib import acn_routing
from .meta_container import MetaContainer
from .meta_ngp import MetaNGP
from .ray_sampling import clamp_rays_near_far, get_ray_directions, get_rays  # noqa: F401  (re-export)
from .trunc_exp import trunc_exp

_LINSPACE_CACHE = {}
_GRAPH_MODE = threading.local()


@contextmanager
def second_order(enabled: bool = True):
    """Within this context, differentiable renders build twice-differentiable graphs (second-order
    MAML: meta_core.py:57 takes ``autograd.grad(create_graph=True)`` of the inner loss): the
    compositing runs as torch ops instead of the HIP forward/backward pair.  Thread-local."""
    prev = getattr(_GRAPH_MODE, "second_order", False)
    _GRAPH_MODE.second_order = bool(enabled)
    try:
        yield
    finally:
        _GRAPH_MODE.second_order = prev


def _second_order() -> bool:
    return getattr(_GRAPH_MODE, "second_order", False)


@contextmanager
def encoding_frozen(enabled: bool = True):
    """Within this context, differentiable single-expert renders evaluate the hash grid without autograd:
    for first-order inner loops (FOMAML / Reptile task_adapt, meta_core.py:14-67), which differentiate
    w.r.t. the fast MLP weights only, the encoding's backward branch (dL/dh0, the table scatter) is dead
    work (the values are unchanged).  The shared background head, not a fast weight either, then runs as
    its fused HIP launch (values within fp32 rounding of the torch chain).  Thread-local."""
    prev = getattr(_GRAPH_MODE, "frozen_encoding", False)
    _GRAPH_MODE.frozen_encoding = bool(enabled)
    try:
        yield
    finally:
        _GRAPH_MODE.frozen_encoding = prev


@contextmanager
def inner_loop_background_cache():
    """Within this context (one first-order task_adapt call), frozen-encoding renders reuse the background
    head's output for rays they have already rendered: the head is not a fast weight and the support rays do
    not change between inner steps, so steps 2..n would recompute the same values (a strided-directions
    copy and a background launch per step).  Entries hold their rays tensor (compared by identity) and end
    with the context.  Only the model's background head is cached ('random' backgrounds are re-drawn per
    render, as in the reference).  Thread-local."""
    prev = getattr(_GRAPH_MODE, "bg_cache", None)
    _GRAPH_MODE.bg_cache = {}
    try:
        yield
    finally:
        _GRAPH_MODE.bg_cache = prev


# Training renders (the differentiable single-expert path: meta inner loops and queries, active_module
# adaptation) visit their rays in direction-cell order (ray_order_kernel, the order render_kernel uses for
# C2): the hash grid's gathers and scatter then see spatially coherent 32-sample tiles.  Every per-ray value is
# computed exactly as before and the outputs are returned in the caller's order, so losses are unchanged; only
# the MLP weight-gradient sums run in another order.  Measured slower on the meta step (66.1 -> 69.2 ms: the
# order launch and the permutations cost more than the gathers gain at 4000-ray tasks), so it
# is off by default; ACN_TRAIN_ORDER=1 turns it on.
TRAIN_RAY_ORDER = os.environ.get("ACN_TRAIN_ORDER", "0") != "0"
_ORDER_MAX = 8192   # ray_order_kernel's single-workgroup limit (ACN_ORDER_MAX)


def _train_order(rays: Tensor):
    """(order, inverse) int64 permutations of ``rays`` by direction cell, through the inner-loop cache when open
    (the support rays are rendered at every inner step)."""
    cache = getattr(_GRAPH_MODE, "bg_cache", None)
    key = ("order", id(rays))
    if cache is not None:
        hit = cache.get(key)
        if hit is not None and hit[0] is rays and hit[1] == rays._version:
            return hit[2], hit[3]
    N = rays.shape[0]
    o32 = torch.empty(N, dtype=torch.int32, device=rays.device)
    from ._lib import check, lib, ptr
    r = rays.contiguous()
    check(lib().acn_ray_order(ptr(r), N, ptr(o32), int(torch.cuda.current_stream(rays.device).cuda_stream)),
          "acn_ray_order")
    order = o32.long()
    inv = torch.empty_like(order)
    inv[order] = torch.arange(N, device=rays.device)
    if cache is not None:
        cache[key] = (rays, rays._version, order, inv)
    return order, inv


def _frozen_background(model, rays, params, rgb_sigma, N, bg_color_default):
    """The background of a frozen-encoding render (no autograd), through the inner-loop cache when open."""
    cache = getattr(_GRAPH_MODE, "bg_cache", None)
    if cache is None or not getattr(model, "use_bg_nerf", False):
        return _get_bg_rgb(model, rays[:, 3:6], params, rgb_sigma, N=N, bg_color_default=bg_color_default)
    key = (id(model), id(rays))
    hit = cache.get(key)
    if hit is not None and hit[0] is rays and hit[1] == rays._version:
        return hit[2]
    bg = _get_bg_rgb(model, rays[:, 3:6], params, rgb_sigma, N=N, bg_color_default=bg_color_default)
    cache[key] = (rays, rays._version, bg)
    return bg


# ============================== BG helpers ===============================
def _get_bg_rgb(model, dirs: Tensor, params, rgb_sigma_or_map, N: int, bg_color_default: str) -> Optional[Tensor]:
    """Background RGB: the model's background head if it has one, else a default colour (:23-45)."""
    if getattr(model, "use_bg_nerf", False):
        return model.background_color(dirs)
    return get_bg_default_color(rgb_sigma_or_map, N, bg_color_default)


def get_bg_default_color(rgb_sigma, N: int, bg_color: str = "white") -> Optional[Tensor]:
    device = None if rgb_sigma is None else rgb_sigma.device
    dtype = None if rgb_sigma is None else rgb_sigma.dtype
    if bg_color == "none":
        return None
    if bg_color == "white":
        return torch.ones(N, 3, device=device, dtype=dtype)
    if bg_color == "black":
        return torch.zeros(N, 3, device=device, dtype=dtype)
    if bg_color == "random":
        return torch.rand(N, 3, device=device, dtype=dtype)
    if bg_color == "last_sample":
        if rgb_sigma is None or rgb_sigma.dim() != 3 or rgb_sigma.size(-1) < 3:
            raise ValueError("bg_color='last_sample' requires rgb_sigma of shape (N,S,4) or (N,S,>=3).")
        return rgb_sigma[:, -1, :3]
    raise ValueError(f"Unknown background policy: {bg_color}")


def apply_bg_mask(rgb_lin: Tensor, mask_invalid: Tensor, policy: str) -> None:
    if not mask_invalid.any():
        return
    policy = str(policy).lower()
    if policy == "white":
        rgb_lin[mask_invalid] = 1.0
    elif policy == "black":
        rgb_lin[mask_invalid] = 0.0
    elif policy == "random":
        n = int(mask_invalid.sum().item())
        rgb_lin[mask_invalid] = torch.rand(n, 3, device=rgb_lin.device, dtype=rgb_lin.dtype)
    elif policy in ("none", "last_sample"):
        pass
    else:
        rgb_lin[mask_invalid] = 1.0


# ============================== Core volume rendering ===============================
def _volume_render_autograd(rgb_sigma, t_vals, bg_rgb, raw_rgb, raw_sigma, sigma_scale):
    """Differentiable compositing, same formulas as ray_rendering.py:137-165 (training path)."""
    rgb = torch.sigmoid(rgb_sigma[..., :3]) if raw_rgb else rgb_sigma[..., :3].clamp(0.0, 1.0)
    sigma = trunc_exp(rgb_sigma[..., 3]) if raw_sigma else rgb_sigma[..., 3].clamp_min(0.0)
    if sigma_scale != 1.0:
        sigma = sigma * float(sigma_scale)
    dists = (t_vals[:, 1:] - t_vals[:, :-1]).clamp_min(1e-4)
    dists = torch.cat([dists, dists[:, -1:]], dim=1)
    alpha = (1.0 - torch.exp(-sigma * dists)).clamp(0.0, 1.0 - 1e-7)
    T = torch.cumprod(torch.cat([torch.ones_like(alpha[:, :1]), 1.0 - alpha + 1e-10], dim=1), dim=1)[:, :-1]
    weights = alpha * T
    rgb_map = (weights.unsqueeze(-1) * rgb).sum(dim=1)
    depth_map = (weights * t_vals).sum(dim=1)
    acc_map = weights.sum(dim=1)
    if bg_rgb is not None:
        rgb_map = rgb_map + (1.0 - acc_map.unsqueeze(-1)) * bg_rgb.to(rgb_map.device, dtype=rgb_map.dtype)
    return rgb_map, depth_map, weights, acc_map


class _VolumeRenderFn(torch.autograd.Function):
    """volume_render with HIP forward (acn_volume_render_fwd) and backward (acn_volume_render_bwd):
    two kernels instead of the ~40 elementwise/scan/reduction launches of the autograd graph."""

    @staticmethod
    def forward(ctx, rgb_sigma, t_vals, bg_rgb, sigma_scale):
        rgb, depth, w, acc = ops.volume_render(rgb_sigma, t_vals, bg_rgb, sigma_scale=sigma_scale)
        # outputs the loss does not use (depth, weights, acc in training) reach backward as None: the
        # kernel treats a NULL output gradient as zero, so autograd need not zero-fill them (3 launches)
        ctx.set_materialize_grads(False)
        ctx.save_for_backward(rgb_sigma, t_vals, bg_rgb)
        ctx.sigma_scale = sigma_scale
        return rgb, depth, w, acc

    @staticmethod
    def backward(ctx, g_rgb, g_depth, g_w, g_acc):
        rgb_sigma, t_vals, bg_rgb = ctx.saved_tensors
        g_rs, g_bg = ops.volume_render_bwd(rgb_sigma, t_vals, bg_rgb, ctx.sigma_scale, g_rgb, g_depth, g_w, g_acc)
        return (g_rs if ctx.needs_input_grad[0] else None, None,
                g_bg if (bg_rgb is not None and ctx.needs_input_grad[2]) else None, None)


def volume_render(rgb_sigma: Tensor, t_vals: Tensor, bg_rgb: Optional[Tensor] = None, *, raw_rgb: bool = False,
                  raw_sigma: bool = False, sigma_scale: float = 1.0, **kwargs) -> Tuple[Tensor, Tensor, Tensor, Tensor]:
    """NeRF compositing: rgb (N,3), depth (N,), weights (N,S), acc (N,) (ray_rendering.py:114-165)."""
    if torch.is_grad_enabled() and (rgb_sigma.requires_grad or (bg_rgb is not None and bg_rgb.requires_grad)):
        if rgb_sigma.is_cuda and not raw_rgb and not raw_sigma and rgb_sigma.dtype == torch.float32 \
                and not _second_order():
            bg = None if bg_rgb is None else bg_rgb.to(rgb_sigma.device, torch.float32)
            return _VolumeRenderFn.apply(rgb_sigma, t_vals, bg, float(sigma_scale))
        return _volume_render_autograd(rgb_sigma, t_vals, bg_rgb, raw_rgb, raw_sigma, sigma_scale)
    out = ops.volume_render(rgb_sigma, t_vals, bg_rgb, raw_rgb=raw_rgb, raw_sigma=raw_sigma, sigma_scale=sigma_scale)
    return tuple(o.to(rgb_sigma.dtype) for o in out)


# ============================== Stratified rendering ===============================
def _t_lin(S: int, device) -> Tensor:
    """torch.linspace(0,1,S) evaluated on the CPU (the reference's device) then moved."""
    key = (S, str(device))
    if key not in _LINSPACE_CACHE:
        _LINSPACE_CACHE[key] = torch.linspace(0.0, 1.0, S).to(device)
    return _LINSPACE_CACHE[key]


@torch.no_grad()
def stratified_t_vals(near: Tensor, far: Tensor, ray_samples: int, randomized: bool = True,
                      u: Optional[Tensor] = None) -> Tensor:
    """S uniform depths in [near, far], jittered within midpoints when randomized (:262-287).
    ``u`` optionally supplies the (N,S) uniforms of the jitter (for reproducible training)."""
    t_lin = _t_lin(ray_samples, near.device).unsqueeze(0)
    t_vals = near.unsqueeze(1) * (1.0 - t_lin) + far.unsqueeze(1) * t_lin
    if randomized:
        mids = 0.5 * (t_vals[:, :-1] + t_vals[:, 1:])
        low = torch.cat([t_vals[:, :1], mids], dim=1)
        high = torch.cat([mids, t_vals[:, -1:]], dim=1)
        t_vals = low + (high - low) * (torch.rand_like(low) if u is None else u)
    return t_vals


FUSED_TRAIN_SAMPLER = True  # tests switch it off to compare with the composed chain
ROUTED_TRAIN = True         # differentiable routed-container renders on the pair kernels (routed.hip)
ENC_EPS = 1e-6  # MetaNGP.enc_eps (a constant fp32 buffer, meta_ngp.py:155-158), known on the host


def _train_expert(model, active_module):
    """The single MetaNGP a differentiable render evaluates (container + active_module, or a bare
    MetaNGP), when it is the fused configuration; else None."""
    sub = model.submodules[active_module] if isinstance(model, MetaContainer) and active_module is not None else (
        model if isinstance(model, MetaNGP) else None)
    return sub if sub is not None and sub._fusable else None


class _BlendFn(torch.autograd.Function):
    """MetaContainer.forward's weighted index_add_ over experts (meta_container.py:300-337) on the
    (sample, expert) pairs: y (P,4) -> (M,4); backward dY_p = dY_m * w_p."""

    @staticmethod
    def forward(ctx, y, pw, pmap, pidx):
        ctx.save_for_backward(pw, pidx)
        return ops.routed_blend_fwd(y, pw, pmap)

    @staticmethod
    def backward(ctx, g):
        pw, pidx = ctx.saved_tensors
        return ops.routed_blend_bwd(g.contiguous(), pidx, pw), None, None, None


def _routed_train_ok(model, rays, active_module) -> bool:
    return (ROUTED_TRAIN and isinstance(model, MetaContainer) and active_module is None and rays.is_cuda
            and rays.dtype == torch.float32 and all(s._fusable for s in model.submodules) and not _second_order())


def _render_routed(model, rays: Tensor, S: int, params, u: Optional[Tensor], bg_color_default: str, sigma_scale):
    """Differentiable render of the routed container (training / runtime_adapt, ray_rendering.py:290-345
    over MetaContainer.forward :275-343): routing + per-expert pair lists on the GPU (routed.hip, one
    host sync for the segment sizes), per expert the HIP hash grid (autograd to its table) and the fused
    MLP, the weighted blend in expert order, HIP compositing.  Experts no sample reaches get no
    gradient at all (grad None), as in the reference's loop."""
    N = rays.shape[0]
    if model.training and u is None:
        u = torch.rand_like(rays.new_empty(N, S))  # the reference's rand_like(low) draw
    boxes = [sub._host_box() for sub in model.submodules]
    t_vals, starts, pidx, pw, x01, sh, pmap = ops.routed_pairs(
        rays.contiguous(), S, u if model.training else None, model.routing_spec(), [b[0] for b in boxes],
        [b[1] for b in boxes], ENC_EPS)
    from .meta_ngp import _FusedMLPFn
    sub_params = model._sub_params(params)
    outs = []
    for k, sub in enumerate(model.submodules):
        a, b = starts[k], starts[k + 1]
        if b == a:
            continue
        h0 = sub.xyz_encoder(x01[a:b])
        ws = [t.contiguous() for t in sub._mlp_tensors(sub_params[k]).values()]
        outs.append(_FusedMLPFn.apply(h0.contiguous(), sh[a:b], *ws))
    y = torch.cat(outs, 0) if len(outs) > 1 else (outs[0] if outs else rays.new_zeros(0, 4))
    rgb_sigma = _BlendFn.apply(y, pw, pmap, pidx).view(N, S, 4)
    bg_rgb = _get_bg_rgb(model, rays[:, 3:6], params, rgb_sigma, N=N, bg_color_default=bg_color_default)
    return volume_render(rgb_sigma, t_vals, bg_rgb=bg_rgb, raw_rgb=False, raw_sigma=False, sigma_scale=sigma_scale)


def _fused_experts(model, params, active_module):
    """(specs, routing) for the fused kernels, or None if the model/config is not fusable."""
    if isinstance(model, MetaContainer):
        if not all(s._fusable for s in model.submodules):
            return None
        if active_module is not None:
            sub = model.submodules[active_module]
            if sub.uses_grad(params):
                return None
            r = acn_routing()
            r.K, r.cluster_2d, r.boundary_margin = 1, 1, 1.0
            spec = sub.expert_spec(params)
            return [spec], r, sub.packed_weights(spec, r, params)
        if model.uses_grad(params):
            return None
        specs, routing = model.expert_specs(params), model.routing_spec()
        return specs, routing, model.packed_weights(specs, routing, None, params)
    if isinstance(model, MetaNGP):
        if not model._fusable or model.uses_grad(params):
            return None
        r = acn_routing()
        r.K, r.cluster_2d, r.boundary_margin = 1, 1, 1.0
        spec = model.expert_spec(params)
        return [spec], r, model.packed_weights(spec, r, params)
    return None


def _fused_background(model, bg_color_default: str, N: int, device):
    """(acn_background, keep) or None when the policy needs the composed path."""
    if getattr(model, "use_bg_nerf", False):
        if torch.is_grad_enabled() and any(p.requires_grad for p in model.bg_mlp.parameters()):
            return None
        return model.background_spec()
    if bg_color_default == "white":
        return ops.make_background("const", color=(1.0, 1.0, 1.0))
    if bg_color_default == "black":
        return ops.make_background("const", color=(0.0, 0.0, 0.0))
    if bg_color_default == "none":
        return ops.make_background("none")
    return None  # "random" / "last_sample": composed path


def render_rays_stratified(model, rays: Tensor, ray_samples: int, params=None, active_module: Optional[int] = None,
                           bg_color_default: str = "white", chunk: int = 1_000_000, sigma_scale=1.0, **kwargs):
    """Stratified renderer: rgb (N,3), depth (N,), weights (N,S), acc (N,) (:290-345)."""
    tau = float(kwargs.get("early_stop_tau", 0.0))
    want_weights = bool(kwargs.get("_want_weights", True))  # render_image drops the (N,S) weights
    N = rays.shape[0]
    if rays.is_cuda:
        fe = _fused_experts(model, params, active_module)
        fb = _fused_background(model, bg_color_default, N, rays.device) if fe is not None else None
        if fe is not None and fb is not None:
            specs, routing, packed = fe
            bg, keep = fb
            jitter = None
            if model.training:
                ju = kwargs.get("jitter_u")
                jitter = ju.to(rays.device, torch.float32).contiguous() if ju is not None else \
                    torch.rand(N, ray_samples, device=rays.device)
            rgb, depth, w, acc = ops.render_stratified(rays, ray_samples, specs, routing,
                                                       0 if len(specs) == 1 else None, bg,
                                                       sigma_scale=float(sigma_scale), tau=tau, jitter=jitter,
                                                       packed=packed, want_weights=want_weights)
            return (rgb.to(rays.dtype), depth.to(rays.dtype), None if w is None else w.to(rays.dtype),
                    acc.to(rays.dtype))
    sub = _train_expert(model, active_module) if FUSED_TRAIN_SAMPLER else None
    if sub is not None and rays.is_cuda and rays.dtype == torch.float32 and sub._fused_train_ok(rays):
        # differentiable single-expert path (training, inner loops): one sampler launch (t-values,
        # unit-box points, SH), the HIP hash grid under autograd and the fused MLP -- the same values
        # as the composed chain below
        from .meta_ngp import _FusedMLPFn
        u = kwargs.get("jitter_u")
        if model.training and u is None:
            u = torch.rand_like(rays.new_empty(N, ray_samples))  # the reference's rand_like(low) draw
        mn, ext = sub._host_box()
        rays_in = rays
        order = None
        if TRAIN_RAY_ORDER and 1 < N <= _ORDER_MAX:
            order, inv = _train_order(rays)
            rays = rays.index_select(0, order)
            if u is not None:
                u = u.to(rays.device).index_select(0, order)
        t_vals, x01, sh = ops.sample_stratified(rays, ray_samples, u if model.training else None, mn, ext,
                                                ENC_EPS)
        if getattr(_GRAPH_MODE, "frozen_encoding", False):
            with torch.no_grad():
                h0 = sub.xyz_encoder(x01)
        else:
            h0 = sub.xyz_encoder(x01)
        ws = [t.contiguous() for t in sub._mlp_tensors(params).values()]
        rgb_sigma = _FusedMLPFn.apply(h0.contiguous(), sh, *ws).view(N, ray_samples, 4)
        # the background of the caller's rays (cached per rays tensor), then in the visiting order
        if getattr(_GRAPH_MODE, "frozen_encoding", False):
            with torch.no_grad():  # nor is the shared background head a fast weight: one fused HIP launch
                bg_rgb = _frozen_background(model, rays_in, params, rgb_sigma, N, bg_color_default)
        else:
            bg_rgb = _get_bg_rgb(model, rays_in[:, 3:6], params, rgb_sigma, N=N, bg_color_default=bg_color_default)
        last_sample = not getattr(model, "use_bg_nerf", False) and bg_color_default == "last_sample"
        if order is not None and not last_sample and bg_rgb is not None and torch.is_tensor(bg_rgb) \
                and bg_rgb.dim() == 2 and bg_rgb.shape[0] == N:
            bg_rgb = bg_rgb.index_select(0, order)   # (last_sample reads the visiting-order samples already)
        out = volume_render(rgb_sigma, t_vals, bg_rgb=bg_rgb, raw_rgb=False, raw_sigma=False,
                            sigma_scale=sigma_scale)
        if order is None:
            return out
        return tuple(None if x is None else x.index_select(0, inv) for x in out)   # the caller's order
    if _routed_train_ok(model, rays, active_module):
        return _render_routed(model, rays, ray_samples, params, kwargs.get("jitter_u"), bg_color_default,
                              sigma_scale)
    # composed (differentiable) path -- same structure as the reference
    o, d = rays[:, :3], rays[:, 3:6]
    near, far = rays[:, 6], rays[:, 7]
    t_vals = stratified_t_vals(near, far, ray_samples, randomized=model.training, u=kwargs.get("jitter_u"))
    pts = o.unsqueeze(1) + d.unsqueeze(1) * t_vals.unsqueeze(-1)
    dirs = d.unsqueeze(1).expand_as(pts)
    id6 = torch.cat([pts, dirs], dim=-1).reshape(-1, 6)
    model_eff = model.submodules[active_module] if active_module is not None else model
    outs = [model_eff(id6[s: s + chunk], params=params) for s in range(0, id6.shape[0], chunk)]
    rgb_sigma = torch.cat(outs, dim=0).view(pts.shape[0], pts.shape[1], 4)
    bg_rgb = _get_bg_rgb(model, dirs[:, 0], params, rgb_sigma, N=rgb_sigma.size(0), bg_color_default=bg_color_default)
    return volume_render(rgb_sigma, t_vals, bg_rgb=bg_rgb, raw_rgb=False, raw_sigma=False, sigma_scale=sigma_scale)


# ============================== Occupancy rendering (Soft MoE) ===============================
@torch.no_grad()
def _intersect_rays_aabb(rays: Tensor, scene_box) -> Tensor:
    """(N,) bool: the ray's [near, far] interval meets the box (ray_rendering.py:170-193)."""
    o, d = rays[:, :3], rays[:, 3:6]
    near, far = rays[:, 6:7], rays[:, 7:8]
    eps = 1e-9
    invd = torch.where(torch.abs(d) > eps, 1.0 / d, torch.full_like(d, 1.0 / eps))
    t0 = (scene_box.min.to(rays.device)[None, :] - o) * invd
    t1 = (scene_box.max.to(rays.device)[None, :] - o) * invd
    tmin = torch.minimum(t0, t1).amax(dim=-1, keepdim=True)
    tmax = torch.maximum(t0, t1).amin(dim=-1, keepdim=True)
    return (torch.minimum(tmax, far) > torch.maximum(tmin, near)).squeeze(-1)


@torch.no_grad()
def _merge_segments_union(ray_indices_list, t0_list, t1_list):
    """Per ray, the sorted distinct boundaries of every expert's segments; consecutive pairs become
    the merged segments (ray_rendering.py:196-258).  One HIP K-way merge per ray."""
    if len(t0_list) == 0:
        dev = torch.device("cpu")
        return (torch.zeros(0, dtype=torch.long, device=dev), torch.zeros(0, dtype=torch.float32, device=dev),
                torch.zeros(0, dtype=torch.float32, device=dev))
    n_rays = int(max(int(r.max().item()) for r in ray_indices_list if r.numel()) + 1) \
        if any(r.numel() for r in ray_indices_list) else 0
    lists = []
    for ri, t0, t1 in zip(ray_indices_list, t0_list, t1_list):
        order = torch.argsort(ri, stable=True)  # each list must be ray-major (marching output already is)
        ri, t0, t1 = ri[order], t0[order], t1[order]
        pi = nerfacc.pack_info(ri, n_rays)
        lists.append((pi[:, 0], pi[:, 1], t0, t1))
    mri, m0, m1, _, _ = occ_ops.union(lists, n_rays)
    return mri, m0, m1


def _bg_or_default(model, d, params, rgb_map, N, bg_color_default):
    return _get_bg_rgb(model, d, params, rgb_map, N, bg_color_default)


def _empty_occ_result(model, rays, d, params, N, bg_color_default):
    acc = rays.new_zeros(N)
    bg_rgb = _get_bg_rgb(model, d, params, None, N, bg_color_default)
    if bg_rgb is not None:
        bg_rgb = bg_rgb.to(rays.device)
    weights = torch.zeros(1, 1, device=rays.device, dtype=rays.dtype)
    return bg_rgb, acc.clone(), weights, acc


def _composite_packed(model, rays, d, params, ri, t0, t1, starts, counts, sigma, rgb, t_mid, N, bg_color_default):
    """nerfacc compositing of packed samples under autograd (training path)."""
    if _second_order():
        raise ops.AcnError("second-order (create_graph) gradients through the occupancy renderer are not "
                           "supported (nerfacc's scan backward is first order too)")
    packed = torch.stack([starts, counts], -1)
    weights = nerfacc.render_weight_from_density(t_starts=t0, t_ends=t1, sigmas=sigma, packed_info=packed)[0][..., None]
    w1 = weights.squeeze(-1)
    rgb_map = nerfacc.accumulate_along_rays(w1, rgb, ri, N)
    depth = nerfacc.accumulate_along_rays(w1, t_mid[:, None], ri, N).squeeze(-1)
    acc = nerfacc.accumulate_along_rays(w1, None, ri, N).squeeze(-1)
    bg_rgb = _get_bg_rgb(model, d, params, rgb_map, N, bg_color_default)
    rgb_map = rgb_map + (1.0 - acc)[..., None] * bg_rgb.to(rgb_map.device, rgb_map.dtype)
    return rgb_map, depth, weights, acc


def render_expert_occ(model, rays: Tensor, *, params=None, bg_color_default: str = "white", chunk: int = 1_000_000,
                      render_step_size=None, alpha_thre=None, cone_angle=None, **kwargs):
    """One expert over its occupancy grid: rgb (N,3), depth (N,), weights (M,1), acc (N,)
    (ray_rendering.py:467-558).  Eval: marching + ONE fused HIP render over the packed samples."""
    N = rays.shape[0]
    o, d = rays[:, :3], rays[:, 3:6]
    if getattr(model, "occ_grid", None) is None:
        return None
    ri, t0, t1, starts, counts = model._occupancy_marching_packed(
        rays, params=params, render_step_size=render_step_size, alpha_thre=alpha_thre, cone_angle=cone_angle)
    if t0.numel() == 0:
        return _empty_occ_result(model, rays, d, params, N, bg_color_default)
    if rays.is_cuda:
        fe = _fused_experts(model, params, None)
        fb = _fused_background(model, bg_color_default, N, rays.device) if fe is not None else None
        if fe is not None and fb is not None:
            specs, routing, packed = fe
            bg, keep = fb
            rgb, depth, w, acc = occ_ops.render_packed(rays, starts, counts, t0, t1, specs, routing, 0, bg,
                                                       packed=packed)
            return rgb.to(rays.dtype), depth.to(rays.dtype), w.to(rays.dtype)[:, None], acc.to(rays.dtype)
    t_mid = 0.5 * (t0 + t1)
    x = o[ri] + d[ri] * t_mid[:, None]
    ds = d[ri]
    outs = [model(torch.cat([x[s:s + chunk], ds[s:s + chunk]], dim=-1), params=params)
            for s in range(0, x.shape[0], chunk)]
    out = torch.cat(outs, 0)
    return _composite_packed(model, rays, d, params, ri, t0, t1, starts, counts, out[:, 3], out[:, :3], t_mid, N,
                             bg_color_default)


def render_rays_occ(model, rays: Tensor, *, params=None, bg_color_default: str = "white", chunk: int = 1_000_000,
                    render_step_size=None, alpha_thre=None, cone_angle=None, active_module: Optional[int] = None,
                    **kwargs):
    """Occupancy-guided soft Mixture-of-Experts renderer (ray_rendering.py:349-464): per expert,
    AABB prefilter + marching over its grid; per-ray boundary union; experts evaluated at the
    midpoints where their routing weight exceeds 1e-8; sigma and rgb blended BEFORE one nerfacc
    integration.  Eval runs marching (HIP), union (HIP) and ONE fused render launch.

    The reference routes the midpoints with ``model._routing(x_mid.view(1, -1, 3))``, which its own
    ``_routing`` rejects (``assert pts.dim() == 2``, meta_container.py:111), so its container path
    raises AssertionError whenever it runs; this build routes the (M, 3) midpoints, the evident
    intent (documented in DESIGN.md)."""
    N = rays.shape[0]
    o, d = rays[:, :3], rays[:, 3:6]
    if active_module is not None:
        sub = model.submodules[active_module]
        return render_expert_occ(sub, rays, params=params, bg_color_default=bg_color_default, chunk=chunk,
                                 render_step_size=render_step_size, alpha_thre=alpha_thre, cone_angle=cone_angle)
    K = len(model.submodules)
    training = any(sub.training for sub in model.submodules)
    lists, any_samples = [], False
    for k, expert in enumerate(model.submodules):
        p_k = model.get_subdict(params, f"submodules.{k}") if params is not None else None
        box = [float(v) for v in torch.cat([expert.scene_box.min, expert.scene_box.max]).tolist()]
        if training:  # subset marching, exactly like the reference (the jitter draws one uniform per hit ray)
            hit = _intersect_rays_aabb(rays, expert.scene_box)
            hit_idx = hit.nonzero(as_tuple=False).squeeze(1)
            if hit_idx.numel() == 0:
                continue
            ri_k, t0_k, t1_k, _, _ = expert._occupancy_marching_packed(
                rays[hit_idx], params=p_k, render_step_size=render_step_size, alpha_thre=alpha_thre,
                cone_angle=cone_angle)
            if t0_k.numel() == 0:
                continue
            g = hit_idx[ri_k]
            pi = nerfacc.pack_info(g, N)
            lists.append((pi[:, 0], pi[:, 1], t0_k, t1_k))
        else:  # eval: the prefilter runs inside the traversal kernel over all rays
            ri_k, t0_k, t1_k, st_k, ct_k = expert._occupancy_marching_packed(
                rays, params=p_k, render_step_size=render_step_size, alpha_thre=alpha_thre, cone_angle=cone_angle,
                prefilter_aabb=box)
            if t0_k.numel() == 0:
                continue
            lists.append((st_k, ct_k, t0_k, t1_k))
        any_samples = True
    if not any_samples:
        return _empty_occ_result(model, rays, d, params, N, bg_color_default)
    mri, m0, m1, mst, mct = occ_ops.union(lists, N)
    if m0.numel() == 0:
        return _empty_occ_result(model, rays, d, params, N, bg_color_default)
    if rays.is_cuda:
        fe = _fused_experts(model, params, None)
        fb = _fused_background(model, bg_color_default, N, rays.device) if fe is not None else None
        if fe is not None and fb is not None:
            specs, routing, packed = fe
            bg, keep = fb
            rgb, depth, w, acc = occ_ops.render_packed(rays, mst, mct, m0, m1, specs, routing,
                                                       0 if K == 1 else None, bg, packed=packed)
            return rgb.to(rays.dtype), depth.to(rays.dtype), w.to(rays.dtype)[:, None], acc.to(rays.dtype)
    # composed (differentiable) path -- the reference's structure
    M = m0.numel()
    t_mid = 0.5 * (m0 + m1)
    x_mid = o[mri] + d[mri] * t_mid[:, None]
    d_mid = d[mri]
    with torch.no_grad():
        W, hard = model._routing(x_mid.view(-1, 3))
        if W is None:
            W = x_mid.new_zeros(M, K)
            W[torch.arange(M, device=W.device), hard.view(-1)] = 1.0
    eps = 1e-8
    SIG = x_mid.new_zeros(M, K)
    RGB = x_mid.new_zeros(M, K, 3)
    for k, expert in enumerate(model.submodules):
        mask = W[:, k] > eps
        if not mask.any():
            continue
        idx = torch.nonzero(mask, as_tuple=False).squeeze(1)
        xb, db = x_mid[idx], d_mid[idx]
        p_k = model.get_subdict(params, f"submodules.{k}") if params is not None else None
        sig_l, rgb_l = [], []
        for s in range(0, idx.numel(), chunk):
            out = expert(torch.cat([xb[s:s + chunk], db[s:s + chunk]], dim=-1), params=p_k)
            rgb_l.append(out[..., :3])
            sig_l.append(out[..., 3])
        SIG = SIG.index_put((idx, torch.full_like(idx, k)), torch.cat(sig_l, 0))
        RGB = RGB.index_put((idx, torch.full_like(idx, k)), torch.cat(rgb_l, 0))
    s_num = (W * SIG).sum(dim=1, keepdim=True).clamp_min(1e-12)
    sigma_mix = s_num.squeeze(1)
    rgb_mix = (W[..., None] * SIG[..., None] * RGB).sum(dim=1) / s_num
    return _composite_packed(model, rays, d, params, mri, m0, m1, mst, mct, sigma_mix, rgb_mix, t_mid, N,
                             bg_color_default)


def render_rays(model, rays, *args, **kwargs):
    """Entry point (:564-574): occupancy renderer once the model's grids are ready, else stratified."""
    if getattr(model, "use_occ", False):
        if not model.occ_ready:
            return render_rays_stratified(model, rays, *args, **kwargs)
        if getattr(model, "warned_occ_ready", False) is False:
            warnings.warn("[OCC] Using nerfacc occupancy renderer (warmup concluded).")
            model.warned_occ_ready = True
        kwargs.pop("ray_samples", None)
        kwargs.pop("_want_weights", None)
        kwargs.pop("sigma_scale", None)
        kwargs.pop("early_stop_tau", None)
        kwargs.pop("jitter_u", None)
        if isinstance(model, MetaNGP):
            return render_expert_occ(model, rays, *args, **kwargs)
        return render_rays_occ(model, rays, *args, **kwargs)
    return render_rays_stratified(model, rays, *args, **kwargs)


@torch.no_grad()
def render_image(model, *, H: int, W: int, fx: float, fy: float, cx: float, cy: float, c2w: Tensor, scene_box,
                 params=None, active_module: Optional[int] = None, ray_samples: int = 64, chunk_points: int = 1 << 16,
                 bg_color_default: str = "white", center_pixels: bool = True, use_amp: bool = False,
                 **kwargs) -> Tuple[Tensor, Optional[Tensor], Optional[Tensor]]:
    """Full frame: per-pixel rays (one fused HIP kernel), render_rays, (H,W,3) clamp (:577-627).
    ``use_amp`` is accepted for interface compatibility; the HIP path computes in fp32."""
    device = next(model.parameters()).device
    rays, _ = ops.get_rays_image(H, W, fx, fy, cx, cy, c2w, scene_box.aabb, device, center_pixels=center_pixels,
                                 near_far_override=(None, None), apply_clamp=True)
    rgb_lin, depth, _, acc = render_rays(model, rays, ray_samples=ray_samples, params=params,
                                         active_module=active_module, bg_color_default=bg_color_default,
                                         chunk=chunk_points, _want_weights=False, **kwargs)
    rgb_lin = rgb_lin.view(H, W, 3).float().clamp_(0, 1)
    return rgb_lin, (None if depth is None else depth.view(-1)), (None if acc is None else acc.view(-1))
