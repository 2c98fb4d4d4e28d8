"""One expert per GPU: the expert-parallel layout of the routed container.

The reference evaluates the K experts of a MetaContainer one after the other in one process
(models/inr/meta_container.py:300-337: per expert nonzero -> index_select -> expert -> index_add_,
routing :97-134) and its online stage adapts all of them together (pipelines/online_stage/
runtime_adapt.py:286-309).  Here expert k lives on the rank ``owner[k]`` (contiguous blocks: rank r
owns experts [r K / W, (r+1) K / W)), every rank holds a shard of the rays, and the only exchange is
per-sample records:

    rank r: its rays -> t values + routed (sample, expert) pairs, grouped by expert in sample order
            (routed.hip) -> 24-B records xd = [world point, ray direction] of every pair
    all-to-all #1 (forward):  records to the owner of the pair's expert (+ the expert id)
    owner:  its experts' fields on the records it received (the same per-expert forward as one GPU)
    all-to-all #2:           (rgb, sigma) 16 B back, in the sender's pair order
    rank r: blend sum_k y_k w_k in expert order, background, compositing -> its rays' pixels
    backward (training): all-to-all #2's backward sends dL/d(rgb, sigma) 16 B to the owners; expert
            gradients are complete on the owner, the replicated background head's gradients are
            all-reduced (SUM: every rank holds part of the batch) and the clip norm is global.

Each expert therefore sees exactly the samples the single-process container routes to it, in the
same order (contiguous ray shards in rank order), so the update equals the single-process one up to
fp32 summation order.  The compute is a ``backend``: ``HipBackend`` runs the HIP kernels; tests plug
a CPU restatement in to check the data movement over gloo.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Optional, Sequence

import torch
import torch.distributed as dist
from torch import Tensor

from .color_space import color_space_transformer


def world_rank(group=None):
    if dist.is_available() and dist.is_initialized():
        return dist.get_world_size(group), dist.get_rank(group)
    return 1, 0


def expert_owner(K: int, world: int) -> List[int]:
    """owner[k]: rank r owns the contiguous experts [r K / W, (r+1) K / W) (sorted-by-expert pair lists
    are then sorted by destination)."""
    return [min(world - 1, (k * world) // K) for k in range(K)]


@dataclass
class PairSet:
    """Routed pairs of a ray shard: t (N,S); counts[k] pairs of expert k, grouped by expert in sample
    order; pidx / pw / pk per pair; xd (P,6) records; pmap (N*S, K) pair index or -1."""
    t: Tensor
    counts: List[int]
    pidx: Tensor
    pw: Tensor
    xd: Tensor
    pmap: Tensor
    pk: Tensor


def _a2a(x: Tensor, out_splits: Sequence[int], in_splits: Sequence[int], group) -> Tensor:
    world, _ = world_rank(group)
    if world == 1:
        return x.clone()
    out = x.new_empty((int(sum(out_splits)),) + tuple(x.shape[1:]))
    dist.all_to_all_single(out, x.contiguous(), list(map(int, out_splits)), list(map(int, in_splits)), group=group)
    return out


class _AllToAll(torch.autograd.Function):
    """all_to_all_single with its transpose as the backward (dL/d(rgb, sigma) back to the owners)."""

    @staticmethod
    def forward(ctx, x, out_splits, in_splits, group):
        ctx.splits, ctx.group = (list(out_splits), list(in_splits)), group
        return _a2a(x, out_splits, in_splits, group)

    @staticmethod
    def backward(ctx, g):
        out_splits, in_splits = ctx.splits
        return _a2a(g.contiguous(), in_splits, out_splits, ctx.group), None, None, None


def exchange_counts(send: Sequence[int], device, group=None) -> List[int]:
    world, _ = world_rank(group)
    if world == 1:
        return list(send)
    s = torch.tensor(list(send), dtype=torch.int64, device=device)
    r = torch.empty_like(s)
    dist.all_to_all_single(r, s, group=group)
    return [int(v) for v in r.cpu().tolist()]


def ep_field(backend, rays: Tensor, S: int, u: Optional[Tensor], K: int, group=None):
    """The routed container's field on this rank's rays with the experts distributed: returns
    (rgb_sigma (N,S,4) blended, PairSet).  Collective: every rank of ``group`` must call it."""
    world, rank = world_rank(group)
    owner = expert_owner(K, world)
    ps = backend.pairs(rays, S, u)
    send = [sum(ps.counts[k] for k in range(K) if owner[k] == r) for r in range(world)]
    recv = exchange_counts(send, rays.device, group)
    payload = torch.cat([ps.xd, ps.pk.to(ps.xd.dtype).unsqueeze(1)], 1)
    got = _a2a(payload, recv, send, group)
    rk = got[:, 6].round().long()
    y_recv = got.new_zeros(got.shape[0], 4)
    for k in range(K):
        if owner[k] != rank:
            continue
        rows = (rk == k).nonzero(as_tuple=False).squeeze(1)   # source-rank order, then sample order
        if rows.numel() == 0:
            continue
        y_recv = y_recv.index_copy(0, rows, backend.expert(k, got.index_select(0, rows)[:, :6].contiguous()))
    if torch.is_grad_enabled() and not y_recv.requires_grad:
        y_recv = y_recv.detach().requires_grad_()   # every rank takes part in the backward exchange
    y = _AllToAll.apply(y_recv, send, recv, group)
    N = rays.shape[0]
    return backend.blend(y, ps).view(N, S, 4), ps


def render_rays_expert_parallel(backend, rays: Tensor, S: int, K: int, group=None, u: Optional[Tensor] = None):
    """render_rays (ray_rendering.py:290-345) of this rank's rays through the expert-parallel container:
    (rgb (N,3), depth (N,), weights (N,S), acc (N,))."""
    rs, ps = ep_field(backend, rays, S, u, K, group)
    return backend.composite(rs, ps.t, rays)


def adapt_step_expert_parallel(P, backend, rays: Tensor, rgbs: Tensor, optimizer, K: int, n_rays_global: int,
                               shared: Sequence[Tensor], grad_clip: Optional[float] = 1.0, group=None,
                               u: Optional[Tensor] = None) -> Tensor:
    """One runtime_adapt update (runtime_adapt.py:286-309, routed container, no active_module) with the
    experts distributed: this rank holds a shard of the global batch of ``n_rays_global`` rays; its owned
    experts get the complete gradients of the samples routed to them from every rank; the ``shared``
    background head is all-reduced; the clip norm is global (shared parameters counted once).  Returns the
    global MSE (device)."""
    from .optim import FusedAdam
    world, _ = world_rank(group)
    optimizer.zero_grad()
    rgb = render_rays_expert_parallel(backend, rays, S=int(P.ray_samples), K=K, group=group, u=u)[0]
    pred, gt = color_space_transformer(rgb, rgbs, color_space=P.color_space)
    loss = ((pred - gt) ** 2).sum() / float(n_rays_global * pred.shape[-1])
    loss.backward()
    if world > 1:
        grads = [p.grad for p in shared if p.grad is not None]
        if grads:
            flat = torch.cat([g.reshape(-1) for g in grads])
            dist.all_reduce(flat, group=group)
            off = 0
            for g in grads:
                g.copy_(flat[off: off + g.numel()].view_as(g))
                off += g.numel()
    if isinstance(optimizer, FusedAdam):
        optimizer.shared_params = {id(p) for p in shared}
        optimizer.step(max_norm=grad_clip, sumsq_group=group)
    else:
        if grad_clip is not None:
            optimizer.last_norm = global_clip_grad_norm_(
                [p for g in optimizer.param_groups for p in g["params"]], shared, grad_clip, group)
        optimizer.step()
    out = loss.detach().clone()
    if world > 1:
        dist.all_reduce(out, group=group)
    return out


def global_clip_grad_norm_(params, shared, max_norm: float, group=None):
    """clip_grad_norm_ over parameters distributed across ranks: each rank's own gradients once, the
    replicated ``shared`` ones once; returns (total_norm, coefficient).  (FusedAdam.step does the same on
    the device with ``sumsq_group``.)"""
    world, _ = world_rank(group)
    sid = {id(p) for p in shared}
    params = [p for p in params if p.grad is not None]
    own = torch.zeros((), dtype=torch.float64, device=params[0].grad.device if params else "cpu")
    for p in params:
        if id(p) not in sid:
            own = own + p.grad.double().pow(2).sum()
    if world > 1:
        dist.all_reduce(own, group=group)
    for p in params:
        if id(p) in sid:
            own = own + p.grad.double().pow(2).sum()
    total = float(own.sqrt())
    coef = min(1.0, max_norm / (total + 1e-6))
    for p in params:
        p.grad.mul_(coef)
    return total, coef


class HipBackend:
    """The compute of the expert-parallel layout on the HIP kernels, for a MetaContainer ``model``
    (every rank holds the container; only the owned experts are evaluated / trained here)."""

    def __init__(self, model, bg_color_default: str = "white"):
        self.model = model
        self.bg_color_default = bg_color_default

    def pairs(self, rays: Tensor, S: int, u: Optional[Tensor]) -> PairSet:
        from . import ops
        m = self.model
        if m.training and u is None:
            u = torch.rand_like(rays.new_empty(rays.shape[0], S))  # the reference's rand_like(low) draw
        t, counts, pidx, pw, xd, pmap, pk = ops.routed_pairs_xd(rays.contiguous(), S, u if m.training else None,
                                                                m.routing_spec())
        return PairSet(t, counts, pidx, pw, xd, pmap, pk)

    def expert(self, k: int, xd: Tensor) -> Tensor:
        from . import ops
        from .meta_ngp import _FusedMLPFn
        from .ray_rendering import ENC_EPS
        sub = self.model.submodules[k]
        if not sub.uses_grad():
            return sub(xd)   # the fused MFMA field kernel (eval)
        mn, ext = sub._host_box()
        x01, sh = ops.xd_unit_sh(xd, mn, ext, ENC_EPS)
        h0 = sub.xyz_encoder(x01)
        ws = [t.contiguous() for t in sub._mlp_tensors(None).values()]
        return _FusedMLPFn.apply(h0.contiguous(), sh, *ws)

    def blend(self, y: Tensor, ps: PairSet) -> Tensor:
        from .ray_rendering import _BlendFn
        return _BlendFn.apply(y.contiguous(), ps.pw, ps.pmap, ps.pidx)

    def composite(self, rs: Tensor, t: Tensor, rays: Tensor):
        from .ray_rendering import _get_bg_rgb, volume_render
        bg = _get_bg_rgb(self.model, rays[:, 3:6], None, rs, N=rays.shape[0], bg_color_default=self.bg_color_default)
        return volume_render(rs, t, bg_rgb=bg, raw_rgb=False, raw_sigma=False)


@torch.no_grad()
def render_image_expert_parallel(model, *, H: int, W: int, fx: float, fy: float, cx: float, cy: float, c2w: Tensor,
                                 scene_box, ray_samples: int = 64, center_pixels: bool = True,
                                 gt_srgb: Optional[Tensor] = None, metrics_space: str = "linear", group=None,
                                 backend=None, rays: Optional[Tensor] = None):
    """render_image (ray_rendering.py:577-627) with the experts distributed: rank r renders a contiguous
    band of the frame's pixels through render_rays_expert_parallel (its samples' records go to the
    experts' owners), then the rendered rows are all-gathered and the PSNR all-reduced (parallel.py).
    Returns (rgb (H,W,3) clamped, depth (H*W,), acc (H*W,), psnr or None)."""
    from .parallel import contiguous_plan, gather_rendered, local_sse, psnr_reduce
    world, rank = world_rank(group)
    if rays is None:
        from . import ops
        device = next(model.parameters()).device
        rays, _ = ops.get_rays_image(H, W, fx, fy, cx, cy, c2w, scene_box.aabb, device, center_pixels=center_pixels,
                                     near_far_override=(None, None), apply_clamp=True)
    backend = backend or HipBackend(model)
    plan = contiguous_plan(rays.shape[0], world, rays.device)
    idx = plan.indices(rank).to(rays.device)
    rgb, depth, _, acc = render_rays_expert_parallel(backend, rays[idx].contiguous(), ray_samples,
                                                     len(model.submodules), group)
    local = torch.cat([rgb.float().view(-1, 3), depth.float().view(-1, 1), acc.float().view(-1, 1)], dim=1)
    full = gather_rendered(local, plan, group)
    rgb_img = full[:, :3].reshape(H, W, 3).clamp_(0, 1)
    psnr = None
    if gt_srgb is not None:
        sse, cnt = local_sse(rgb_img.view(-1, 3)[idx], gt_srgb.to(rgb_img.device).view(-1, 3)[idx], metrics_space)
        psnr = psnr_reduce(sse, cnt, rgb_img.device, group)
    return rgb_img, full[:, 3], full[:, 4], psnr
