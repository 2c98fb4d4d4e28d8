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

from typing import Optional, Tuple

import torch
from torch import Tensor

from . import ops
from ._lib import acn_routing
from .meta_container import MetaContainer
from .meta_ngp import MetaNGP
from .ray_sampling import clamp_rays_near_far, get_ray_directions, get_rays  # noqa: F401  (re-export)
from .trunc_exp import trunc_exp

_LINSPACE_CACHE = {}


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
        if rgb_sigma.is_cuda and not raw_rgb and not raw_sigma and rgb_sigma.dtype == torch.float32:
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


def render_rays(model, rays, *args, **kwargs):
    """Entry point (:564-574).  The occupancy renderer is not part of this build."""
    if getattr(model, "use_occ", False):
        raise NotImplementedError("occupancy-grid rendering (nerfacc) is not part of this build (SURVEY §8(f))")
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
