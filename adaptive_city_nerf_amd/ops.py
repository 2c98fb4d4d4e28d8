"""Tensor-level wrappers over libacnerf.so (include/acnerf.h).

Each function validates shapes the way the reference's asserts do, makes inputs contiguous fp32
device tensors, allocates outputs with the caching allocator and launches on the current stream.
No CPU path exists: CPU tensors raise.
"""
from __future__ import annotations

import ctypes as C
import os
from typing import Dict, Optional, Sequence

import torch

from . import _lib
from ._lib import (ACN_BG_CONST, ACN_BG_MLP, ACN_BG_NONE, AcnError, acn_background, acn_expert,
                   acn_routing, check, ptr, require_hip, stream_of)

MLP_KEYS = (
    ("sig_w0", "sigma_trunk.0.linear.weight"), ("sig_b0", "sigma_trunk.0.linear.bias"),
    ("sig_w1", "sigma_trunk.1.linear.weight"), ("sig_b1", "sigma_trunk.1.linear.bias"),
    ("sigh_w", "sigma_head.weight"), ("sigh_b", "sigma_head.bias"),
    ("geo_w", "geo_head.weight"), ("geo_b", "geo_head.bias"),
    ("col_w0", "color_mlp.0.linear.weight"), ("col_b0", "color_mlp.0.linear.bias"),
    ("col_w1", "color_mlp.1.linear.weight"), ("col_b1", "color_mlp.1.linear.bias"),
    ("col_w2", "color_mlp.2.weight"), ("col_b2", "color_mlp.2.bias"),
)
MLP_SHAPES = {
    "sigma_trunk.0.linear.weight": (64, 32), "sigma_trunk.0.linear.bias": (64,),
    "sigma_trunk.1.linear.weight": (64, 64), "sigma_trunk.1.linear.bias": (64,),
    "sigma_head.weight": (1, 64), "sigma_head.bias": (1,),
    "geo_head.weight": (15, 64), "geo_head.bias": (15,),
    "color_mlp.0.linear.weight": (64, 31), "color_mlp.0.linear.bias": (64,),
    "color_mlp.1.linear.weight": (64, 64), "color_mlp.1.linear.bias": (64,),
    "color_mlp.2.weight": (3, 64), "color_mlp.2.bias": (3,),
}


def _f32(t: torch.Tensor) -> torch.Tensor:
    return t.detach().to(torch.float32).contiguous()


# ---------------------------------------------------------------------------------------------
def hashgrid_fwd(x01: torch.Tensor, table: torch.Tensor, resolutions: Sequence[int], log2T: int,
                 F: int, interp: int) -> torch.Tensor:
    require_hip(x01, "HashGridEncoder")
    assert x01.shape[-1] == 3, f"Expected (...,3), got {tuple(x01.shape)}"
    L = len(resolutions)
    x = _f32(x01).view(-1, 3)
    tab = _f32(table)
    if tab.shape != (L << log2T, F):
        raise AcnError(f"hash table must be ({L << log2T}, {F}), got {tuple(tab.shape)}")
    out = torch.empty(x.shape[0], L * F, device=x.device, dtype=torch.float32)
    res = (C.c_int32 * L)(*[int(r) for r in resolutions])
    check(_lib.lib().acn_hashgrid_fwd(ptr(x), x.shape[0], ptr(tab), res, L, log2T, F, interp, ptr(out),
                                      stream_of(x)), "acn_hashgrid_fwd")
    return out.view(*x01.shape[:-1], L * F)


# workspace cap of the deterministic hash-grid backward (~24 B x 8 x L per point, 3 GB at 1M points)
DET_WS_CAP = 1 << 30


def hashgrid_bwd(x01: torch.Tensor, grad_out: torch.Tensor, resolutions: Sequence[int], log2T: int, F: int,
                 interp: int, deterministic: Optional[bool] = None, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Table gradient (scatter-add).  ``deterministic`` (default: torch.are_deterministic_algorithms_enabled())
    selects the sort-based backward (acn_hashgrid_bwd_det: bitwise reproducible, every row summed in point
    order) over the float-atomic one.  ``out``: an existing (L * 2^log2T, F) fp32 buffer the float-atomic
    scatter adds into (accumulation; the deterministic backward accumulates into it too, each row continuing
    its serial sum).  The deterministic workspace (records + sort buffers, ~3 KB per point at L = 16) is
    bounded by processing the points in chunks of at most DET_WS_CAP bytes: the kernel adds every row's
    contributions, in point order, onto the row's current value, so consecutive chunks give exactly the
    serial sum of one pass."""
    L = len(resolutions)
    x = _f32(x01).view(-1, 3)
    g = _f32(grad_out).view(-1, L * F)
    if out is not None:
        if tuple(out.shape) != (L << log2T, F) or out.dtype != torch.float32 or not out.is_contiguous():
            raise ValueError("hashgrid_bwd: out must be a contiguous fp32 (L * 2^log2T, F) buffer")
    gt = out if out is not None else torch.zeros(L << log2T, F, device=x.device, dtype=torch.float32)
    res = (C.c_int32 * L)(*[int(r) for r in resolutions])
    if deterministic is None:
        deterministic = torch.are_deterministic_algorithms_enabled()
    if deterministic and F == 2:
        L_ = _lib.lib()
        M = x.shape[0]
        per = max(1, int(L_.acn_hashgrid_bwd_det_workspace_bytes(1 << 16, L, log2T, interp)) >> 16)
        chunk = max(1, min(M, DET_WS_CAP // per))
        ws = torch.empty(max(int(L_.acn_hashgrid_bwd_det_workspace_bytes(chunk, L, log2T, interp)), 1),
                         dtype=torch.uint8, device=x.device)
        for m0 in range(0, M, chunk):
            n = min(chunk, M - m0)
            check(L_.acn_hashgrid_bwd_det(ptr(x[m0:m0 + n]), n, ptr(g[m0:m0 + n]), res, L, log2T, F, interp, ptr(gt),
                                          ptr(ws), ws.numel(), stream_of(x)), "acn_hashgrid_bwd_det")
        return gt
    check(_lib.lib().acn_hashgrid_bwd(ptr(x), x.shape[0], ptr(g), res, L, log2T, F, interp, ptr(gt),
                                      stream_of(x)), "acn_hashgrid_bwd")
    return gt


def sh_fwd(d: torch.Tensor, levels: int) -> torch.Tensor:
    require_hip(d, "SHEncoder")
    assert d.shape[-1] == 3, f"Expected (...,3); got {tuple(d.shape)}"
    x = _f32(d).view(-1, 3)
    out = torch.empty(x.shape[0], levels * levels, device=x.device, dtype=torch.float32)
    check(_lib.lib().acn_sh_fwd(ptr(x), x.shape[0], levels, ptr(out), stream_of(x)), "acn_sh_fwd")
    return out.view(*d.shape[:-1], levels * levels)


# ---------------------------------------------------------------------------------------------
class ExpertSpec:
    """The device-side description of one MetaNGP expert: hash table + level resolutions + AABB +
    the 14 MLP tensors (module parameters or fast weights from a `params` dict)."""

    def __init__(self, table: torch.Tensor, resolutions: Sequence[int], log2T: int, interp: int,
                 aabb_min: Sequence[float], aabb_extent: Sequence[float], mlp: Dict[str, torch.Tensor],
                 F: int = 2):
        self.keep = []
        s = acn_expert()
        tab = _f32(table)
        self.keep.append(tab)
        s.table = ptr(tab)
        s.L = len(resolutions)
        s.log2T = int(log2T)
        s.F = int(F)
        s.interp = int(interp)
        for i, r in enumerate(resolutions):
            s.res[i] = int(r)
        s.aabb_min[:] = [float(v) for v in aabb_min]
        s.aabb_extent[:] = [float(v) for v in aabb_extent]
        for field, key in MLP_KEYS:
            if key not in mlp:
                raise AcnError(f"missing MLP tensor {key!r}")
            t = _f32(mlp[key])
            if tuple(t.shape) != MLP_SHAPES[key]:
                raise AcnError(f"the fused HIP field supports the reference architecture (nerf_runner.py:102-121); "
                               f"{key} has shape {tuple(t.shape)}, expected {MLP_SHAPES[key]}")
            self.keep.append(t)
            setattr(s, field, ptr(t))
        self.s = s
        self.device = tab.device


def make_routing(centroids: torch.Tensor, K: int, cluster_2d: bool, boundary_margin: float) -> acn_routing:
    r = acn_routing()
    r.K = int(K)
    r.cluster_2d = int(bool(cluster_2d))
    r.boundary_margin = float(boundary_margin)
    c = centroids.detach().float().cpu()
    for k in range(K):
        for a in range(3):
            r.centroids[k][a] = float(c[k, a])
    return r


def make_background(mode: str, color=None, mlp: Optional[Dict[str, torch.Tensor]] = None):
    b = acn_background()
    keep = []
    if mode == "mlp":
        b.mode = ACN_BG_MLP
        w1 = _f32(mlp["0.weight"]); b1 = _f32(mlp["0.bias"]); w2 = _f32(mlp["2.weight"]); b2 = _f32(mlp["2.bias"])
        if w1.shape[1] != 16 or w2.shape[0] != 3:
            raise AcnError("background MLP must be Linear(16, H) -> Linear(H, 3)")
        keep += [w1, b1, w2, b2]
        b.hidden = int(w1.shape[0])
        b.w1, b.b1, b.w2, b.b2 = ptr(w1), ptr(b1), ptr(w2), ptr(b2)
    elif mode == "const":
        b.mode = ACN_BG_CONST
        b.color[:] = [float(v) for v in color]
    else:
        b.mode = ACN_BG_NONE
    return b, keep


def _experts_array(experts: Sequence[ExpertSpec]):
    return (acn_expert * len(experts))(*[e.s for e in experts])


def pack_experts(experts: Sequence[ExpertSpec], routing: acn_routing, active_module: Optional[int] = None,
                 out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """MFMA-ordered weight image of the experts the next fused call evaluates (acn_pack_experts)."""
    K = 1 if active_module is not None else routing.K
    nbytes = int(_lib.lib().acn_workspace_bytes(K))
    dev = experts[0].device
    if out is None or out.numel() * 4 < nbytes or out.device != dev:
        out = torch.empty(nbytes // 4, device=dev, dtype=torch.float32)
    arr = _experts_array(experts)
    check(_lib.lib().acn_pack_experts(arr, C.byref(routing), -1 if active_module is None else int(active_module),
                                      ptr(out), out.numel() * 4, int(torch.cuda.current_stream(dev).cuda_stream)),
          "acn_pack_experts")
    return out


class PackCache:
    """Re-packs only when the (module-owned) weights changed: the key is built from the identity,
    storage and version counter of every packed tensor (in-place updates and load_state_dict bump
    the version).  Fast-weight dicts are never cached (their storage is recycled per step)."""

    def __init__(self):
        self.key = None
        self.ws = None

    def get(self, experts: Sequence[ExpertSpec], routing: acn_routing, active_module: Optional[int], key):
        if key is not None and key == self.key and self.ws is not None:
            return self.ws
        self.ws = pack_experts(experts, routing, active_module, out=self.ws)
        self.key = key
        return self.ws


# Optional timing hook (bench.py): when set to a list, render_stratified / field_fwd append a pair of
# recorded HIP events bracketing exactly the fused kernel on the launch stream.
EVENT_HOOK = None


def field_fwd(x: torch.Tensor, experts: Sequence[ExpertSpec], routing: acn_routing,
              active_module: Optional[int] = None, packed: Optional[torch.Tensor] = None) -> torch.Tensor:
    require_hip(x, "MetaContainer.forward")
    assert x.dim() == 2 and x.shape[-1] >= 6, "x must be (N,D>=6)"
    xx = _f32(x)
    M = xx.shape[0]
    out = torch.empty(M, 4, device=xx.device, dtype=torch.float32)
    if M == 0:
        return out
    ws = packed if packed is not None else pack_experts(experts, routing, active_module)
    arr = _experts_array(experts)
    hook = EVENT_HOOK
    if hook is not None:
        e0 = torch.cuda.Event(enable_timing=True)
        e0.record()
    check(_lib.lib().acn_field_fwd(ptr(xx), M, xx.shape[1], arr, C.byref(routing),
                                   -1 if active_module is None else int(active_module), ptr(ws),
                                   ws.numel() * 4, ptr(out), stream_of(xx)), "acn_field_fwd")
    if hook is not None:
        e1 = torch.cuda.Event(enable_timing=True)
        e1.record()
        hook.append((e0, e1))
    return out



# Default of render_stratified(reorder=None): direction-sorted visiting order for small batches
# (acn_render_stratified_fwd_ordered; outputs are identical either way, only the speed changes).
REORDER = True


def render_stratified(rays: torch.Tensor, S: int, experts: Sequence[ExpertSpec], routing: acn_routing,
                      active_module: Optional[int], background, sigma_scale: float = 1.0, tau: float = 0.0,
                      jitter: Optional[torch.Tensor] = None, want_weights: bool = True,
                      packed: Optional[torch.Tensor] = None, reorder: Optional[bool] = None):
    require_hip(rays, "render_rays")
    assert rays.dim() == 2 and rays.shape[-1] == 8, "rays must be (N,8)"
    r = _f32(rays)
    N = r.shape[0]
    dev = r.device
    rgb = torch.empty(N, 3, device=dev, dtype=torch.float32)
    depth = torch.empty(N, device=dev, dtype=torch.float32)
    acc = torch.empty(N, device=dev, dtype=torch.float32)
    weights = torch.empty(N, S, device=dev, dtype=torch.float32) if want_weights else None
    if N == 0:
        return rgb, depth, weights, acc
    ws = packed if packed is not None else pack_experts(experts, routing, active_module)
    arr = _experts_array(experts)
    jit = None if jitter is None else _f32(jitter)
    # scratch for the ray visiting order (small batches; the outputs do not depend on it)
    obytes = int(_lib.lib().acn_render_order_bytes(N)) if (REORDER if reorder is None else reorder) else 0
    order = torch.empty(obytes // 4, device=dev, dtype=torch.int32) if obytes else None
    hook = EVENT_HOOK
    if hook is not None:
        e0 = torch.cuda.Event(enable_timing=True)
        e0.record()
    check(_lib.lib().acn_render_stratified_fwd_ordered(
        ptr(r), N, int(S), ptr(jit), arr, C.byref(routing), -1 if active_module is None else int(active_module),
        C.byref(background), float(sigma_scale), float(tau), ptr(ws), ws.numel() * 4, ptr(rgb), ptr(depth),
        ptr(weights), ptr(acc), ptr(order), obytes, stream_of(r)), "acn_render_stratified_fwd_ordered")
    if hook is not None:
        e1 = torch.cuda.Event(enable_timing=True)
        e1.record()
        hook.append((e0, e1))
    return rgb, depth, weights, acc


def volume_render(rgb_sigma: torch.Tensor, t_vals: torch.Tensor, bg_rgb: Optional[torch.Tensor] = None,
                  raw_rgb: bool = False, raw_sigma: bool = False, sigma_scale: float = 1.0):
    require_hip(rgb_sigma, "volume_render")
    rs = _f32(rgb_sigma)
    t = _f32(t_vals)
    N, S = t.shape
    assert rs.shape == (N, S, 4), f"rgb_sigma must be (N,S,4), got {tuple(rs.shape)}"
    dev = rs.device
    bg = None if bg_rgb is None else _f32(bg_rgb.to(dev)).view(N, 3)
    rgb = torch.empty(N, 3, device=dev, dtype=torch.float32)
    depth = torch.empty(N, device=dev, dtype=torch.float32)
    w = torch.empty(N, S, device=dev, dtype=torch.float32)
    acc = torch.empty(N, device=dev, dtype=torch.float32)
    check(_lib.lib().acn_volume_render_fwd(ptr(rs), ptr(t), ptr(bg), N, S, int(raw_rgb), int(raw_sigma),
                                           float(sigma_scale), ptr(rgb), ptr(depth), ptr(w), ptr(acc),
                                           stream_of(rs)), "acn_volume_render_fwd")
    return rgb, depth, w, acc


def volume_render_bwd(rgb_sigma: torch.Tensor, t_vals: torch.Tensor, bg_rgb: Optional[torch.Tensor], sigma_scale: float,
                      g_rgb, g_depth, g_weights, g_acc):
    """dL/d(rgb_sigma), dL/d(bg) of volume_render (raw flags off) for the given output gradients."""
    rs = _f32(rgb_sigma)
    t = _f32(t_vals)
    N, S = t.shape
    dev = rs.device
    bg = None if bg_rgb is None else _f32(bg_rgb.to(dev)).view(N, 3)
    gr = None if g_rgb is None else _f32(g_rgb).view(N, 3)
    gd = None if g_depth is None else _f32(g_depth).view(N)
    gw = None if g_weights is None else _f32(g_weights).view(N, S)
    ga = None if g_acc is None else _f32(g_acc).view(N)
    g_rs = torch.empty(N, S, 4, device=dev, dtype=torch.float32)
    g_bg = torch.empty(N, 3, device=dev, dtype=torch.float32) if bg is not None else None
    check(_lib.lib().acn_volume_render_bwd(ptr(rs), ptr(t), ptr(bg), N, S, float(sigma_scale), ptr(gr), ptr(gd),
                                           ptr(gw), ptr(ga), ptr(g_rs), ptr(g_bg), stream_of(rs)),
          "acn_volume_render_bwd")
    return g_rs, g_bg


def mse_linear_fwd(pred: torch.Tensor, gt: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """compute_mse_loss's loss in color_space 'linear' (acn_mse_linear_fwd): a 0-d device tensor (written into
    ``out``, a one-element fp32 tensor on the same device, when given)."""
    p, g = _f32(pred).reshape(-1), _f32(gt).reshape(-1)
    if p.numel() != g.numel() or p.numel() == 0:
        raise ValueError(f"mse_linear: pred / gt sizes {p.numel()} / {g.numel()}")
    if out is None:
        out = torch.empty((), device=p.device, dtype=torch.float32)
    elif out.numel() != 1 or out.dtype != torch.float32 or out.device != p.device:
        raise ValueError("mse_linear_fwd: out must be a one-element fp32 tensor on the inputs' device")
    ws = _mse_ws(p.device)
    check(_lib.lib().acn_mse_linear_fwd_ws(ptr(p), ptr(g), p.numel(), ptr(out), ptr(ws), ws.numel(), stream_of(p)),
          "acn_mse_linear_fwd_ws")
    return out


_MSE_WS = {}


def _mse_ws(device) -> torch.Tensor:
    """Zeroed workspace of acn_mse_linear_fwd_ws per (device, stream): its ticket counter returns to 0
    after every call, so one buffer serves every later call on that stream.  Under stream capture every
    captured call gets a workspace of its own: graphs captured on torch's shared capture stream would
    otherwise share one ticket counter, and two of them replayed concurrently would race on it."""
    if torch.cuda.is_current_stream_capturing():
        ws = torch.zeros(int(_lib.lib().acn_mse_linear_workspace_bytes()), dtype=torch.uint8, device=device)
        return _lib.capture_keepalive(ws)   # lives as long as the graph it is baked into
    key = (device, int(torch.cuda.current_stream(device).cuda_stream))
    ws = _MSE_WS.get(key)
    if ws is None:
        ws = _MSE_WS[key] = torch.zeros(int(_lib.lib().acn_mse_linear_workspace_bytes()), dtype=torch.uint8,
                                        device=device)
    return ws


def mse_linear_bwd(pred: torch.Tensor, gt: torch.Tensor, g_loss: torch.Tensor) -> torch.Tensor:
    p, g = _f32(pred).reshape(-1), _f32(gt).reshape(-1)
    gl = _f32(g_loss.reshape(1))
    out = torch.empty_like(p)
    check(_lib.lib().acn_mse_linear_bwd(ptr(p), ptr(g), p.numel(), ptr(gl), ptr(out), stream_of(p)),
          "acn_mse_linear_bwd")
    return out.view(pred.shape)


def get_rays_image(H: int, W: int, fx: float, fy: float, cx: float, cy: float, c2w: torch.Tensor,
                   aabb: Optional[torch.Tensor], device, center_pixels: bool = True, near: Optional[float] = None,
                   far: Optional[float] = None, near_far_override=None, apply_clamp: bool = True):
    c = c2w.detach().float().cpu().contiguous()[:3, :4].contiguous()
    c_arr = (C.c_float * 12)(*c.view(-1).tolist())
    a_arr = None
    if aabb is not None:
        a = aabb.detach().float().cpu().contiguous().view(-1)
        a_arr = (C.c_float * 6)(*a.tolist())
    hn = hf = 0
    nv = fv = 0.0
    if near_far_override is not None:
        if near_far_override[0] is not None:
            hn, nv = 1, float(near_far_override[0])
        if near_far_override[1] is not None:
            hf, fv = 1, float(near_far_override[1])
    rays = torch.empty(H * W, 8, device=device, dtype=torch.float32)
    valid = torch.empty(H * W, device=device, dtype=torch.uint8)
    check(_lib.lib().acn_get_rays(int(H), int(W), float(fx), float(fy), float(cx), float(cy), int(center_pixels),
                                  c_arr, a_arr, float(near or 0.0), float(far or 0.0), hn, nv, hf, fv,
                                  int(apply_clamp), ptr(rays), ptr(valid), stream_of(rays)), "acn_get_rays")
    return rays, valid.bool()


def _host_f32(t, n):
    v = t.detach().float().cpu().contiguous().view(-1)
    if v.numel() != n:
        raise AcnError(f"expected {n} values, got {v.numel()}")
    return (C.c_float * n)(*v.tolist())


def ray_directions(H: int, W: int, fx: float, fy: float, cx: float, cy: float, center_pixels: bool, device):
    dirs = torch.empty(H, W, 3, device=device, dtype=torch.float32)
    check(_lib.lib().acn_ray_directions(int(H), int(W), float(fx), float(fy), float(cx), float(cy),
                                        int(center_pixels), ptr(dirs), stream_of(dirs)), "acn_ray_directions")
    return dirs


def rays_from_dirs(dirs: torch.Tensor, c2w: torch.Tensor, aabb: Optional[torch.Tensor], near_c: float = 0.0,
                   far_c: float = 0.0, eps: float = 1e-8, max_bound: float = 1e10, invalid_value: float = 1e10):
    require_hip(dirs, "get_rays")
    d = _f32(dirs).view(-1, 3)
    rays = torch.empty(d.shape[0], 8, device=d.device, dtype=torch.float32)
    c = _host_f32(c2w[:3, :4], 12)
    a = None if aabb is None else _host_f32(aabb, 6)
    check(_lib.lib().acn_rays_from_dirs(ptr(d), d.shape[0], c, a, float(near_c), float(far_c), float(eps),
                                        float(max_bound), float(invalid_value), ptr(rays), stream_of(d)),
          "acn_rays_from_dirs")
    return rays


def ray_aabb(origins: torch.Tensor, dirs: torch.Tensor, aabb: torch.Tensor, eps: float, max_bound: float,
             invalid_value: float):
    require_hip(origins, "SceneBox.ray_aabb_intersect")
    o = _f32(origins).view(-1, 3)
    d = _f32(dirs.to(o.device)).view(-1, 3)
    tmin = torch.empty(o.shape[0], device=o.device, dtype=torch.float32)
    tmax = torch.empty_like(tmin)
    check(_lib.lib().acn_ray_aabb(ptr(o), ptr(d), o.shape[0], _host_f32(aabb, 6), float(eps), float(max_bound),
                                  float(invalid_value), ptr(tmin), ptr(tmax), stream_of(o)), "acn_ray_aabb")
    return tmin, tmax


def clamp_rays(rays: torch.Tensor, near_far_override, eps: float = 1e-6, invalid_value: float = float("inf")):
    """Returns (rays', valid).  rays' is a new tensor unless override is None (then rays itself)."""
    require_hip(rays, "clamp_rays_near_far")
    apply = near_far_override is not None
    r = _f32(rays).clone() if apply else _f32(rays)
    hn = hf = 0
    nv = fv = 0.0
    if apply:
        if near_far_override[0] is not None:
            hn, nv = 1, float(near_far_override[0])
        if near_far_override[1] is not None:
            hf, fv = 1, float(near_far_override[1])
    valid = torch.empty(r.shape[0], device=r.device, dtype=torch.uint8)
    check(_lib.lib().acn_clamp_rays(ptr(r), r.shape[0], int(apply), hn, nv, hf, fv, float(eps), float(invalid_value),
                                    ptr(valid), stream_of(r)), "acn_clamp_rays")
    return (r if apply else rays), valid.bool()


def routing_fwd(pts: torch.Tensor, routing: acn_routing):
    require_hip(pts, "MetaContainer._routing")
    p = _f32(pts)
    M = p.shape[0]
    if routing.boundary_margin > 1.0:
        W = torch.empty(M, routing.K, device=p.device, dtype=torch.float32)
        check(_lib.lib().acn_routing_fwd(ptr(p), M, p.shape[1], C.byref(routing), ptr(W), None, stream_of(p)),
              "acn_routing_fwd")
        return W, None
    hard = torch.empty(M, device=p.device, dtype=torch.int32)
    check(_lib.lib().acn_routing_fwd(ptr(p), M, p.shape[1], C.byref(routing), None, ptr(hard), stream_of(p)),
          "acn_routing_fwd")
    return None, hard.long()


def background_fwd(dirs: torch.Tensor, background) -> torch.Tensor:
    require_hip(dirs, "MetaContainer.background_color")
    d = _f32(dirs).view(-1, 3)
    out = torch.empty(d.shape[0], 3, device=d.device, dtype=torch.float32)
    check(_lib.lib().acn_background_fwd(ptr(d), d.shape[0], C.byref(background), ptr(out), stream_of(d)),
          "acn_background_fwd")
    return out


def background_bwd(dirs: torch.Tensor, background, g_out: torch.Tensor, grads: Sequence[torch.Tensor]) -> None:
    """Gradients of the MLP background head's four tensors (written into ``grads`` = [gw1, gb1, gw2, gb2],
    overwritten) for dL/d(bg rgb) ``g_out`` (N,3) (acn_background_bwd)."""
    d = _f32(dirs).view(-1, 3)
    g = _f32(g_out).view(-1, 3)
    for t in grads:
        if not (t.is_contiguous() and t.dtype == torch.float32 and t.device == d.device):
            raise AcnError("background_bwd: gradient buffers must be contiguous fp32 on the rays' device")
    L = _lib.lib()
    if torch.cuda.is_current_stream_capturing():   # one workspace per captured call (see _mse_ws)
        ws = _lib.capture_keepalive(torch.empty(int(L.acn_background_bwd_workspace_bytes()), dtype=torch.uint8,
                                                device=d.device))
    else:
        key = (d.device, int(torch.cuda.current_stream(d.device).cuda_stream))
        ws = _BG_WS.get(key)
        if ws is None:
            ws = _BG_WS[key] = torch.empty(int(L.acn_background_bwd_workspace_bytes()), dtype=torch.uint8,
                                           device=d.device)
    check(L.acn_background_bwd(ptr(d), d.shape[0], C.byref(background), ptr(g), *[ptr(t) for t in grads], ptr(ws),
                               ws.numel(), stream_of(d)), "acn_background_bwd")


_BG_WS = {}


# ------------------------------------------------------------------------------------------
# expert MLP of the training path (mlp_train.hip)
MLP_SAVE_COLS, MLP_GRAD_COLS = 325, 275


def _mlp_struct(ws: Sequence[torch.Tensor]):
    from ._lib import acn_mlp
    w = acn_mlp()
    for name, t in zip(("w0", "b0", "w1", "b1", "wsh", "bsh", "wg", "bg", "wc0", "bc0", "wc1", "bc1", "wc2", "bc2"), ws):
        if not (t.is_contiguous() and t.dtype == torch.float32):
            raise AcnError(f"mlp_train: {name} must be a contiguous fp32 tensor")
        setattr(w, name, t.data_ptr())
    return w


MLP_GROUP = 2048


def _mlp_ws(device):
    return torch.empty(int(mlp_fn("acn_mlp_workspace_bytes")()), dtype=torch.uint8, device=device)


def _fm_zeros(M: int, cols: int, device) -> torch.Tensor:
    """(groups, cols, 2048) feature-major buffer; only the last group's tail needs zeros."""
    G = (M + MLP_GROUP - 1) // MLP_GROUP
    t = torch.empty(G, cols, MLP_GROUP, device=device, dtype=torch.float32)
    if M % MLP_GROUP:
        t[-1, :, M % MLP_GROUP:].zero_()
    return t


def mlp_train_fwd(h0: torch.Tensor, sh: torch.Tensor, ws: Sequence[torch.Tensor], save: bool = True,
                  precision: Optional[str] = None, return_img: bool = False):
    """(M,32) hash features + (M,16) SH -> out (M,4) and the feature-major saved layer inputs (or None);
    with ``return_img`` also the call's packed weight image (for mlp_train_bwd_dw(img=...))."""
    require_hip(h0, "MetaNGP MLP (training)")
    M = h0.shape[0]
    out = torch.empty(M, 4, device=h0.device, dtype=torch.float32)
    sv = _fm_zeros(M, MLP_SAVE_COLS, h0.device) if save else None
    w = _mlp_struct(ws)
    img = torch.empty(int(mlp_fn("acn_mlp_workspace_bytes", precision)()), dtype=torch.uint8, device=h0.device)
    check(mlp_fn("acn_mlp_train_fwd", precision)(ptr(h0), ptr(sh), M, C.byref(w), ptr(out),
                                                  ptr(sv) if save else None, ptr(img), stream_of(h0)),
          "acn_mlp_train_fwd")
    if return_img:
        return out, sv, (img if M > 0 else None)
    return out, sv


def mlp_train_bwd(save: torch.Tensor, out: torch.Tensor, gout: torch.Tensor, ws: Sequence[torch.Tensor],
                  want_h0: bool = True):
    M = out.shape[0]
    gs = _fm_zeros(M, MLP_GRAD_COLS, out.device)
    gh = torch.empty(M, 32, device=out.device, dtype=torch.float32) if want_h0 else None
    w = _mlp_struct(ws)
    check(mlp_fn("acn_mlp_train_bwd")(ptr(save), ptr(out), ptr(gout), M, C.byref(w), ptr(gs),
                                       ptr(gh) if want_h0 else None, ptr(_mlp_ws(out.device)), stream_of(out)),
          "acn_mlp_train_bwd")
    return gs, gh


# [dW | db] layout of acn_mlp_train_bwd_dw (include/acnerf.h): the 14 gradients, acn_mlp order
MLP_DW_SHAPES = ((64, 32), (64,), (64, 64), (64,), (1, 64), (1,), (15, 64), (15,), (64, 31), (64,), (64, 64), (64,),
                 (3, 64), (3,))
MLP_DW_FLOATS = 13715
# Precision of the training MLP's layer products: "fp16x3" (default: the fp32-accurate 3-term fp16 split on
# v_mfma_f32_32x32x16_f16), "fp32" (exact fp32 MFMA, the acn_mlp_*_exact entry points) or "amp" (the
# reference's use_amp=True arithmetic: torch.autocast(float16) -- one fp16 product per term, fp16 layer outputs
# and gradients; the acn_mlp_*_amp entry points; pair it with a loss scale, see optim.AmpScaler).  Env ACN_TRAIN_MLP.
TRAIN_MLP_PRECISION = os.environ.get("ACN_TRAIN_MLP", "fp16x3")
_MLP_SUFFIX = {"fp16x3": "", "fp32": "_exact", "amp": "_amp"}


def set_train_mlp_precision(mode: str) -> None:
    """Select the training MLP kernels ("fp16x3", "fp32" or "amp") for later calls; step objects
    (RoutedAdaptStep, ExpertParallelAdaptStep) keep the precision they were built with."""
    global TRAIN_MLP_PRECISION
    if mode not in _MLP_SUFFIX:
        raise ValueError(f"train MLP precision must be one of {sorted(_MLP_SUFFIX)}, got {mode!r}")
    TRAIN_MLP_PRECISION = mode


def mlp_fn(name: str, precision: Optional[str] = None):
    """The training-MLP entry point ``name`` of the selected precision."""
    return getattr(_lib.lib(), name + _MLP_SUFFIX[precision or TRAIN_MLP_PRECISION])
# Optional timing hook (bench.py --workload meta): when set to a list, every acn_mlp_train_bwd_dw call appends
# (start event, end event, M, want_h0) recorded on the current stream around the call (weight pack +
# mlp_bwd_dw_kernel + mlp_dw_reduce_kernel)
DW_HOOK = None
# Algorithmic MACs per sample of the fused MLP backward (SURVEY §8(d) MLP shapes): dW = every weight
# (32x64 + 64x64 + 64x[15|1] + 31x64 + 64x64 + 64x3 = 13,440); dX = the layer-input gradients the chain
# needs (64x3 + 64x64 + 64x15 geo columns + 64x16 heads + 64x64 = 10,368, + 32x64 when dL/dh0 is wanted).
# The in-register forward recompute (13,440 MACs) is extra work of this design, not counted.
MLP_BWD_MACS_DW, MLP_BWD_MACS_DX, MLP_BWD_MACS_DX0, MLP_FWD_MACS = 13440, 10368, 2048, 13440


def mlp_bwd_flops(M: int, want_h0: bool) -> int:
    """Algorithmic FLOPs (2 per MAC) of one fused MLP backward over M samples: dW + dX, no recompute."""
    return 2 * M * (MLP_BWD_MACS_DW + MLP_BWD_MACS_DX + (MLP_BWD_MACS_DX0 if want_h0 else 0))


def mlp_train_bwd_dw(h0: torch.Tensor, sh: torch.Tensor, out: torch.Tensor, gout: torch.Tensor,
                     ws: Sequence[torch.Tensor], want_h0: bool = True, img: Optional[torch.Tensor] = None,
                     precision: Optional[str] = None):
    """Fused backward: the 14 weight / bias gradients (views of one flat buffer, nn.Linear shapes) and
    dL/dh0 (M, 32) or None, from h0 / sh (the forward is re-run in registers) and dL/dout.  ``img``: the
    packed image mlp_train_fwd(return_img=True) returned for the same weights and precision (the
    backward then skips its own pack)."""
    require_hip(h0, "MetaNGP MLP (training)")
    M = out.shape[0]
    dw = torch.empty(MLP_DW_FLOATS, device=out.device, dtype=torch.float32)
    gh = torch.empty(M, 32, device=out.device, dtype=torch.float32) if want_h0 else None
    wsp = torch.empty(int(mlp_fn("acn_mlp_dw_workspace_bytes", precision)()), dtype=torch.uint8, device=out.device)
    hook = DW_HOOK
    if hook is not None:
        e0 = torch.cuda.Event(enable_timing=True)
        e0.record()
    if img is not None:
        check(mlp_fn("acn_mlp_train_bwd_dw_img", precision)(ptr(h0), ptr(sh), ptr(out), ptr(gout), M, ptr(img),
                                                             ptr(dw), ptr(gh) if want_h0 else None, ptr(wsp),
                                                             stream_of(out)), "acn_mlp_train_bwd_dw_img")
    else:
        w = _mlp_struct(ws)
        check(mlp_fn("acn_mlp_train_bwd_dw", precision)(ptr(h0), ptr(sh), ptr(out), ptr(gout), M, C.byref(w),
                                                         ptr(dw), ptr(gh) if want_h0 else None, ptr(wsp),
                                                         stream_of(out)), "acn_mlp_train_bwd_dw")
    if hook is not None:
        e1 = torch.cuda.Event(enable_timing=True)
        e1.record()
        hook.append((e0, e1, int(M), bool(want_h0)))
    grads, o = [], 0
    for shp in MLP_DW_SHAPES:
        n = 1
        for d in shp:
            n *= d
        grads.append(dw[o:o + n].view(shp))
        o += n
    return grads, gh


def sample_stratified(rays: torch.Tensor, S: int, jitter: Optional[torch.Tensor], aabb_min, aabb_extent,
                      eps: float):
    """Training-path sampler (acn_sample_stratified): t_vals (N,S), x01 (N*S,3) in the expert's unit box
    clamped to [eps, 1 - eps] with eps the fp32 enc_eps buffer (1 - eps evaluated in fp32, as
    MetaNGP._world_to_unit's tensor arithmetic does), SH (N*S,16)."""
    require_hip(rays, "render_rays_stratified sampler")
    rays = rays.contiguous()
    N = rays.shape[0]
    dev = rays.device
    t = torch.empty(N, S, device=dev, dtype=torch.float32)
    x01 = torch.empty(N * S, 3, device=dev, dtype=torch.float32)
    sh = torch.empty(N * S, 16, device=dev, dtype=torch.float32)
    jit = None
    if jitter is not None:
        jitter = jitter.to(dev, torch.float32).contiguous()
        jit = ptr(jitter)
    mn = (C.c_float * 3)(*aabb_min)
    ex = (C.c_float * 3)(*aabb_extent)
    import numpy as np
    lo = np.float32(eps)
    hi = np.float32(1.0) - lo
    check(_lib.lib().acn_sample_stratified(ptr(rays), N, int(S), jit, C.cast(mn, C.c_void_p), C.cast(ex, C.c_void_p),
                                           C.c_float(lo), C.c_float(hi),
                                           ptr(t), ptr(x01), ptr(sh), stream_of(rays)), "acn_sample_stratified")
    return t, x01, sh


# ------------------------------------------------------------------------------------------
# routed container, differentiable path (routed.hip)
def routed_pairs(rays: torch.Tensor, S: int, jitter: Optional[torch.Tensor], routing: acn_routing, aabb_mins,
                 aabb_exts, eps: float):
    """t_vals (N,S) and the (sample, expert) pairs of the routed container: returns (t_vals, starts (K+1
    host ints), pidx (P,) int32, pw (P,), x01 (P,3), sh (P,16), pmap (M,K) int32).  One host
    synchronisation (the segment sizes) sits between the count and the scatter launches."""
    require_hip(rays, "render_rays (routed container)")
    r = _f32(rays)
    N = r.shape[0]
    M = N * int(S)
    K = int(routing.K)
    dev = r.device
    L = _lib.lib()
    ws = torch.empty(int(L.acn_routed_workspace_bytes(M, K)), dtype=torch.uint8, device=dev)
    t = torch.empty(N, int(S), device=dev, dtype=torch.float32)
    starts = torch.empty(2 * K + 1, device=dev, dtype=torch.int64)
    jit = None if jitter is None else _f32(jitter.to(dev))
    check(L.acn_routed_count(ptr(r), N, int(S), ptr(jit), C.byref(routing), 1, ptr(t), ptr(starts), ptr(ws),
                             ws.numel(), stream_of(r)), "acn_routed_count")
    st = [int(v) for v in starts[: K + 1].cpu().tolist()]
    P = st[K]
    pidx = torch.empty(P, device=dev, dtype=torch.int32)
    pw = torch.empty(P, device=dev, dtype=torch.float32)
    x01 = torch.empty(P, 3, device=dev, dtype=torch.float32)
    sh = torch.empty(P, 16, device=dev, dtype=torch.float32)
    pmap = torch.empty(M, K, device=dev, dtype=torch.int32)
    mins = (C.c_float * (3 * K))(*[float(v) for row in aabb_mins for v in row])
    exts = (C.c_float * (3 * K))(*[float(v) for row in aabb_exts for v in row])
    import numpy as np
    lo = np.float32(eps)
    hi = np.float32(1.0) - lo
    check(L.acn_routed_scatter(ptr(r), N, int(S), K, ptr(t), ptr(starts), C.cast(mins, C.c_void_p),
                               C.cast(exts, C.c_void_p), C.c_float(lo), C.c_float(hi), 1, ptr(ws), ptr(pidx),
                               ptr(pw), ptr(x01), ptr(sh), ptr(pmap), None, stream_of(r)), "acn_routed_scatter")
    return t, st, pidx, pw, x01, sh, pmap


def routed_blend_fwd(y: torch.Tensor, pw: torch.Tensor, pmap: torch.Tensor) -> torch.Tensor:
    M, K = pmap.shape
    out = torch.empty(M, 4, device=pmap.device, dtype=torch.float32)
    yy = _f32(y).view(-1, 4) if y.numel() else None
    check(_lib.lib().acn_routed_blend_fwd(ptr(yy), ptr(pw), ptr(pmap), M, K, ptr(out), stream_of(pmap)),
          "acn_routed_blend_fwd")
    return out


def routed_blend_bwd(g: torch.Tensor, pidx: torch.Tensor, pw: torch.Tensor,
                     live: Optional[torch.Tensor] = None) -> torch.Tensor:
    """dY per pair slot; ``live``: a device int64 holding the live slot count (capacity-sized buffers),
    slots past it are left unwritten."""
    P = pidx.shape[0]
    gy = torch.empty(P, 4, device=pidx.device, dtype=torch.float32)
    check(_lib.lib().acn_routed_blend_bwd(ptr(_f32(g)), ptr(pidx), ptr(pw), P, ptr(live), ptr(gy), stream_of(pidx)),
          "acn_routed_blend_bwd")
    return gy


def routed_pairs_xd(rays: torch.Tensor, S: int, jitter: Optional[torch.Tensor], routing: acn_routing,
                    tile_rays: int = 0):
    """t_vals (N,S) and the routed pairs as expert-parallel records: (t_vals, counts (K host ints), pidx, pw,
    xd (P,6) world point + direction, pmap (M,K), pk (P,)); pairs grouped by expert, in sample order, or with
    ``tile_rays`` > 0 in depth tiles of that many rays (acn_routed_*_tiled, the ExpertParallelRenderer order)."""
    require_hip(rays, "expert-parallel render")
    r = _f32(rays)
    N = r.shape[0]
    M = N * int(S)
    K = int(routing.K)
    dev = r.device
    L = _lib.lib()
    ws = torch.empty(int(L.acn_routed_workspace_bytes(M, K)), dtype=torch.uint8, device=dev)
    t = torch.empty(N, int(S), device=dev, dtype=torch.float32)
    seg = torch.empty(2 * K + 1, device=dev, dtype=torch.int64)
    jit = None if jitter is None else _f32(jitter.to(dev))
    check(L.acn_routed_count(ptr(r), N, int(S), ptr(jit), C.byref(routing), 1, ptr(t), ptr(seg), ptr(ws),
                             ws.numel(), stream_of(r)), "acn_routed_count")
    sh = [int(v) for v in seg.cpu().tolist()]
    counts = sh[K + 1:]
    P = sh[K]
    pidx = torch.empty(P, device=dev, dtype=torch.int32)
    pw = torch.empty(P, device=dev, dtype=torch.float32)
    xd = torch.empty(P, 6, device=dev, dtype=torch.float32)
    pk = torch.empty(P, device=dev, dtype=torch.int32)
    pmap = torch.empty(M, K, device=dev, dtype=torch.int32)
    if tile_rays:   # the same segments (capacities = the counts), laid out in depth-tile order
        check(L.acn_routed_count_caps_tiled(ptr(r), N, int(S), ptr(jit), C.byref(routing), (C.c_int64 * K)(*counts),
                                            int(tile_rays), ptr(t), ptr(seg), ptr(ws), ws.numel(), stream_of(r)),
              "acn_routed_count_caps_tiled")
    check(L.acn_routed_scatter_xd_tiled(ptr(r), N, int(S), K, int(tile_rays), ptr(t), ptr(seg), ptr(ws), ptr(pidx),
                                        ptr(pw), ptr(xd), ptr(pmap), ptr(pk), stream_of(r)),
          "acn_routed_scatter_xd_tiled")
    return t, counts, pidx, pw, xd, pmap, pk


def xd_unit_sh(xd: torch.Tensor, aabb_min, aabb_extent, eps: float):
    """Owner side: (P,6) records -> x01 (P,3) in the expert's unit box and SH-4 (P,16) of the direction."""
    require_hip(xd, "expert-parallel expert")
    x = _f32(xd)
    P = x.shape[0]
    x01 = torch.empty(P, 3, device=x.device, dtype=torch.float32)
    sh = torch.empty(P, 16, device=x.device, dtype=torch.float32)
    mn = (C.c_float * 3)(*aabb_min)
    ex = (C.c_float * 3)(*aabb_extent)
    import numpy as np
    lo = np.float32(eps)
    hi = np.float32(1.0) - lo
    check(_lib.lib().acn_xd_unit_sh(ptr(x), P, C.cast(mn, C.c_void_p), C.cast(ex, C.c_void_p), C.c_float(lo),
                                    C.c_float(hi), ptr(x01), ptr(sh), stream_of(x)), "acn_xd_unit_sh")
    return x01, sh
