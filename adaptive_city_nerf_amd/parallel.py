"""Multi-GPU rendering: one process per GPU over RCCL.

The reference renders on one device (nerfs/ray_rendering.py:577-627 ``render_image``;
pipelines/online_stage/runtime_adapt.py:120-172 evaluates PSNR per image).  Rays are independent,
so the frame is split over ranks with every expert replicated (K x 128 MiB is nothing against
288 GB of HBM) and no collective in the data path; the only exchanges are

* one ``all_gather_into_tensor`` of the rendered rows (rgb, depth, acc: 20 B per ray), and
* one ``all_reduce`` of two fp64 numbers (sum of squared error, element count) for the PSNR.

Shard plan.  ``"expert"`` (default) sorts the rays by the expert that owns their midpoint (the
hard routing rule of MetaContainer._routing, meta_container.py:97-134) and cuts the sorted list
into equal contiguous chunks: every rank renders the same number of rays (balanced), and its
samples hit one or two experts, so the hash tables a GPU touches stay resident in its 256 MiB
Infinity Cache instead of K tables thrashing it (SURVEY §7 "sparse hash traffic").
``"rows"`` gives rank r a contiguous band of pixel rows (the plain tile split).

Both are exact: each ray is rendered by exactly one rank with the full soft-routed container, so
the gathered frame is bit-identical to a single-GPU ``render_image`` of the same rays.
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Callable, Optional, Tuple

import torch
import torch.distributed as dist
from torch import Tensor

from .color_space import color_space_transformer


FORCE_COLLECTIVES = False   # tests: the all-gather and the PSNR all-reduce through the group even at world size 1


def _world_rank(group) -> Tuple[int, int]:
    if dist.is_available() and dist.is_initialized():
        return dist.get_world_size(group), dist.get_rank(group)
    return 1, 0


@dataclass
class ShardPlan:
    """Rank r renders rays ``perm[r*chunk : min((r+1)*chunk, N)]`` (rank-major permutation)."""
    perm: Tensor
    chunk: int
    N: int
    world: int

    def indices(self, rank: int) -> Tensor:
        lo = min(rank * self.chunk, self.N)
        hi = min(lo + self.chunk, self.N)
        return self.perm[lo:hi]


def contiguous_plan(N: int, world: int, device=None) -> ShardPlan:
    """Equal contiguous chunks in ray order (pixel rows for a frame)."""
    return ShardPlan(torch.arange(N, device=device), max(1, math.ceil(N / world)), N, world)


def expert_sorted_plan(keys: Tensor, world: int) -> ShardPlan:
    """Stable sort by owning expert, then equal chunks: balanced and expert-local."""
    N = keys.numel()
    perm = torch.argsort(keys.view(-1).to(torch.int64), stable=True)
    return ShardPlan(perm, max(1, math.ceil(N / world)), N, world)


def direction_cell(rays: Tensor, bits: int = 6) -> Tensor:
    """Z-order cell of each ray's direction on a 2^bits x 2^bits grid: the gnomonic coordinates
    (d.e1 / d.m, d.e2 / d.m) about the batch's mean direction m (an image-plane position for one
    camera), quantised over their bounding box -- the key ray_order_kernel (render.hip) sorts a
    single-expert batch by.  As a secondary key after the expert it keeps each expert's rays in
    image-region order, so a workgroup's neighbours (and, with XCD bands, an XCD's L2) share the
    mid-level hash cells.  Rays with a zero / non-finite direction get cell 0."""
    d = rays[:, 3:6].double()
    ok = torch.isfinite(d).all(1) & (d.abs().sum(1) > 0)
    dn = torch.where(ok.unsqueeze(1), d / d.norm(dim=1, keepdim=True).clamp_min(1e-300), torch.zeros_like(d))
    m = dn.sum(0)
    if float(m.norm()) == 0.0:
        return torch.zeros(rays.shape[0], dtype=torch.int64, device=rays.device)
    m = m / m.norm()
    a = torch.tensor([1.0, 0.0, 0.0], dtype=d.dtype, device=d.device)
    if abs(float(m[0])) > 0.9:
        a = torch.tensor([0.0, 1.0, 0.0], dtype=d.dtype, device=d.device)
    e1 = torch.linalg.cross(m, a)
    e1 = e1 / e1.norm()
    e2 = torch.linalg.cross(m, e1)
    dm = dn @ m
    front = ok & (dm > 1e-6)
    u = torch.where(front, (dn @ e1) / dm.clamp_min(1e-6), torch.zeros_like(dm))
    v = torch.where(front, (dn @ e2) / dm.clamp_min(1e-6), torch.zeros_like(dm))
    n = 1 << bits

    def q(x):
        lo, hi = float(x[front].min()) if bool(front.any()) else 0.0, float(x[front].max()) if bool(front.any()) else 1.0
        return ((x - lo) / max(hi - lo, 1e-12) * n).floor().clamp(0, n - 1).to(torch.int64)
    qx, qy = q(u), q(v)
    key = torch.zeros_like(qx)
    for b in range(bits):
        key |= ((qx >> b) & 1) << (2 * b) | ((qy >> b) & 1) << (2 * b + 1)
    return torch.where(front, key, torch.zeros_like(key))


def expert_spatial_keys(rays: Tensor, model, bits: int = 6) -> Tensor:
    """Sort key (owning expert, direction cell): ``expert_sorted_plan`` on it groups the rays by
    expert and, within an expert, by image region."""
    return dominant_expert(rays, model).to(torch.int64) * (1 << (2 * bits)) + direction_cell(rays, bits)


def multi_expert_rays(rays: Tensor, model, ray_samples: int) -> Tensor:
    """(N,) bool: rays whose eval-mode samples (stratified, no jitter) reach more than one expert under the
    container's soft routing -- the rays render_slots_kernel evaluates with two or more experts per tile."""
    from . import ops
    S = int(ray_samples)
    _, _, _, _, _, pmap, _ = ops.routed_pairs_xd(rays, S, None, model.routing_spec())
    hit = (pmap.view(rays.shape[0], S, -1) >= 0).any(dim=1)     # (N, K): expert k reached by some sample
    return hit.sum(dim=1) > 1


def dominant_expert(rays: Tensor, model) -> Tensor:
    """Expert owning each ray's midpoint o + d (near + far)/2: argmin centroid distance, the hard
    routing rule of meta_container.py:119-121 (HIP kernel acn_routing_fwd)."""
    from . import ops
    from ._lib import acn_routing
    spec = model.routing_spec()
    r = acn_routing()
    r.K, r.cluster_2d, r.boundary_margin = spec.K, spec.cluster_2d, 1.0  # bm <= 1 -> argmin
    for k in range(spec.K):
        for a in range(3):
            r.centroids[k][a] = spec.centroids[k][a]
    near, far = rays[:, 6], rays[:, 7]
    mid = torch.where(torch.isfinite(far), 0.5 * (near + far), torch.zeros_like(near))
    mid = torch.where(torch.isfinite(mid), mid, torch.zeros_like(mid))
    pts = (rays[:, :3] + rays[:, 3:6] * mid.unsqueeze(1)).contiguous()
    _, hard = ops.routing_fwd(pts, r)
    return hard


def gather_rendered(local: Tensor, plan: ShardPlan, group=None) -> Tensor:
    """All-gather every rank's (n_r, C) rendered rows and undo the plan's permutation -> (N, C)."""
    world, _ = _world_rank(group)
    C = local.shape[1]
    buf = torch.zeros(plan.chunk, C, device=local.device, dtype=local.dtype)
    buf[: local.shape[0]] = local
    if world == 1 and not FORCE_COLLECTIVES:
        full = buf
    elif buf.is_cuda and dist.get_backend(group) == "gloo":
        # gloo has no device all-gather: stage through the host (tests run two ranks on one GPU this way)
        parts = [torch.empty(plan.chunk, C, dtype=local.dtype) for _ in range(world)]
        dist.all_gather(parts, buf.cpu(), group=group)
        full = torch.cat(parts).to(local.device)
    else:
        full = torch.empty(world * plan.chunk, C, device=local.device, dtype=local.dtype)
        dist.all_gather_into_tensor(full, buf, group=group)
    out = torch.empty(plan.N, C, device=local.device, dtype=local.dtype)
    out[plan.perm.to(local.device)] = full[: plan.N]
    return out


def psnr_reduce(sse: float, count: float, device, group=None) -> float:
    """Global PSNR from per-rank sums: -10 log10(clamp_min(SSE/count, 1e-8)) (runtime_adapt.py:156-157)."""
    world, _ = _world_rank(group)
    t = torch.tensor([sse, count], dtype=torch.float64, device=device)
    if world > 1 or FORCE_COLLECTIVES:
        if t.is_cuda and dist.get_backend(group) == "gloo":
            t = t.cpu()
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
    mse = max(float(t[0]) / max(float(t[1]), 1.0), 1e-8)
    return -10.0 * math.log10(mse)


RenderFn = Callable[[Tensor], Tuple[Tensor, Tensor, Tensor]]


def render_rays_sharded(rays: Tensor, render_fn: RenderFn, plan: ShardPlan, group=None) -> Tuple[Tensor, Tensor, Tensor]:
    """Render this rank's share of ``rays`` with ``render_fn(rays) -> (rgb, depth, acc)`` and
    all-gather the full (rgb (N,3), depth (N,), acc (N,)) on every rank."""
    _, rank = _world_rank(group)
    idx = plan.indices(rank).to(rays.device)
    rgb, depth, acc = render_fn(rays[idx].contiguous())
    local = torch.cat([rgb.float().view(-1, 3), depth.float().view(-1, 1), acc.float().view(-1, 1)], dim=1)
    full = gather_rendered(local, plan, group)
    return full[:, :3], full[:, 3], full[:, 4]


def local_sse(pred_lin: Tensor, gt_srgb: Tensor, metrics_space: str) -> Tuple[float, float]:
    """Sum of squared error and element count in the metric colour space (color_space.py:22-66)."""
    p, g = color_space_transformer(pred_lin, gt_srgb, metrics_space)
    d = (p.double() - g.double())
    return float((d * d).sum()), float(d.numel())


@torch.no_grad()
def render_image_sharded(model, *, H: int, W: int, fx: float, fy: float, cx: float, cy: float, c2w: Tensor,
                         scene_box, params=None, active_module: Optional[int] = None, ray_samples: int = 64,
                         bg_color_default: str = "white", center_pixels: bool = True, gt_srgb: Optional[Tensor] = None,
                         metrics_space: str = "linear", shard: str = "expert", group=None,
                         render_fn: Optional[RenderFn] = None, rays: Optional[Tensor] = None, **kwargs):
    """Multi-GPU ``render_image`` (ray_rendering.py:577-627): every rank builds the frame's rays,
    renders its shard, and receives the whole frame.  Returns (rgb (H,W,3) clamped, depth (H*W,),
    acc (H*W,), psnr or None) -- psnr against ``gt_srgb`` (H,W,3) in ``metrics_space`` reduced
    over ranks.  ``render_fn``/``rays`` override the HIP renderer and ray generator (tests)."""
    world, rank = _world_rank(group)
    if rays is None:
        from . import ops
        device = next(model.parameters()).device
        rays, _ = ops.get_rays_image(H, W, fx, fy, cx, cy, c2w, scene_box.aabb, device, center_pixels=center_pixels,
                                     near_far_override=(None, None), apply_clamp=True)
    if render_fn is None:
        from .ray_rendering import render_rays

        def render_fn(r):
            rgb, depth, _, acc = render_rays(model, r, ray_samples=ray_samples, params=params,
                                             active_module=active_module, bg_color_default=bg_color_default,
                                             _want_weights=False, **kwargs)
            return rgb, depth, acc
    if shard == "expert" and world > 1 and hasattr(model, "routing_spec") and active_module is None:
        plan = expert_sorted_plan(dominant_expert(rays, model), world)
    else:
        plan = contiguous_plan(rays.shape[0], world, rays.device)
    rgb, depth, acc = render_rays_sharded(rays, render_fn, plan, group)
    rgb_img = rgb.view(H, W, 3).clamp_(0, 1)
    psnr = None
    if gt_srgb is not None:
        idx = plan.indices(rank).to(rays.device)
        sse, cnt = local_sse(rgb_img.view(-1, 3)[idx], gt_srgb.to(rgb_img.device).view(-1, 3)[idx], metrics_space)
        psnr = psnr_reduce(sse, cnt, rgb_img.device, group)
    return rgb_img, depth, acc, psnr
