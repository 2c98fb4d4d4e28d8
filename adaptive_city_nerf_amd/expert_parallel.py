"""One expert per GPU: the expert-parallel layout of the routed container.

The reference evaluates the K experts of a MetaContainer one after the other in one process
(models/inr/meta_container.py:300-337: per expert nonzero -> index_select -> expert -> index_add_,
routing :97-134) and its online stage adapts all of them together (pipelines/online_stage/
runtime_adapt.py:286-309).  Here expert k lives on the rank ``owner[k]`` (contiguous blocks: rank r
owns experts [r K / W, (r+1) K / W)), every rank holds a shard of the rays, and the only exchange is
per-sample records:

    rank r: its rays -> t values + routed (sample, expert) pairs, grouped by expert in sample order
            (routed.hip; the renderer: in depth tiles of neighbouring rays) -> 24-B records xd = [world
            point, ray direction] of every pair
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

import os
from dataclasses import dataclass
from typing import List, Optional, Sequence

import torch
import torch.distributed as dist
from torch import Tensor

from ._lib import graph_capture
from .color_space import color_space_transformer


# ExpertParallelRenderer's record order: depth tiles of this many neighbouring rays (0: sample order; env
# ACN_EP_TILE overrides).  32: the busiest C4 owner rank at 0.47 of HBM against 0.25 in sample order
EP_TILE_RAYS = 32


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
    from . import ops
    from .optim import FusedAdam
    if ops.TRAIN_MLP_PRECISION == "amp":
        raise ValueError("adapt_step_expert_parallel: the use_amp MLP precision needs a loss scale; select 'fp16x3' "
                         "or 'fp32' for expert-parallel steps")
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


class ExpertParallelRenderer:
    """render_rays (ray_rendering.py:290-345, eval) of this rank's rays through the routed container with the
    experts distributed -- expert k on rank expert_owner(K, W)[k] -- and no host synchronisation: every
    exchange has a constant size, so one call is a fixed sequence of launches and collectives (at world size 1
    the exchanges are copies and ``graph=True`` replays the whole call as one HIP graph).

    Per call, on every rank (batches of up to ``n_rays`` rays):
      sender  t values, routing and (sample, expert) pairs in the fixed layout of acn_routed_count_fixed:
              expert k's pairs at [k C, k C + min(count, C)), 24-B [world point, direction] records -- grouped
              by owner, the pair buffer is the all-to-all send buffer
      a2a #0  the per-expert live counts (int64) to the owners;  a2a #1 the records (constant splits)
      owner   acn_ep_field_fwd: the field of its experts on every received record, written in the received
              layout (no compaction, no scatter-back)
      a2a #2  (rgb, sigma) back to the senders' pair slots
      sender  acn_ep_composite: blend in expert order + background + compositing in one launch -> rgb, depth,
              acc (+ weights): the (N, S, 4) field tensor is never materialised.
    The per-sample arithmetic is the fused routed render's (SH-first colour layer 0), so each ray renders bit
    for bit as in the fused single-process routed render.  ``capacity`` C per (sender, expert) segment:
    n_rays * S (default, never overflows) or smaller to shrink the exchange; ``overflowed()`` reads the counts
    back (one host read, to be called lazily, e.g. once per frame) and a caller re-renders an overflowed batch at
    full capacity.  ``render_planned(rays, counts)``: the exchange sized to the live records -- ``counts`` (W, K)
    are every rank's pair counts of this batch (acn_routed_count_batches, all-gathered once per frame by
    render_rays_ep_batched), the (sender, expert) segments hold exactly those pairs, so the all-to-alls move
    40 B per live pair and nothing else (the reference sends each expert only its routed samples:
    meta_container.py:307-321).  Reference: models/inr/meta_container.py:300-337, nerfs/ray_rendering.py:577-627."""

    def __init__(self, model, n_rays: int, ray_samples: int, group=None, capacity: Optional[int] = None,
                 graph: bool = False, bg_color_default: str = "white", want_weights: bool = False,
                 tile_rays: Optional[int] = None):
        from . import _lib, ops
        from ._lib import AcnError
        from .meta_container import MetaContainer
        from .ray_rendering import _fused_background
        if not isinstance(model, MetaContainer) or not all(s._fusable for s in model.submodules):
            raise AcnError("ExpertParallelRenderer: a MetaContainer of reference-configuration experts is required")
        self.comm = comm = _Comm(group)
        W, rank = comm.world, comm.rank
        self.model, self.group = model, group
        K = len(model.submodules)
        owner = expert_owner(K, W)
        own = [k for k in range(K) if owner[k] == rank]
        if not own:
            raise AcnError(f"ExpertParallelRenderer: rank {rank} owns no expert (K = {K} < W = {W})")
        E = len(own)
        eo = [owner.count(o) for o in range(W)]
        N, S = int(n_rays), int(ray_samples)
        M = N * S
        Cc = int(capacity) if capacity is not None else M
        if Cc < 1:
            raise AcnError("ExpertParallelRenderer: capacity must be >= 1")
        self.K, self.E, self.W, self.N, self.S, self.M, self.C = K, E, W, N, S, M, Cc
        # the order of every expert's records: depth tiles of tile_rays neighbouring rays (acn_routed_*_tiled), so
        # the owner's waves see neighbouring points; 0: sample order.  Results go back by position,
        # so the order changes no value.
        self.tile_rays = int(os.environ.get("ACN_EP_TILE", EP_TILE_RAYS) if tile_rays is None else tile_rays)
        if self.tile_rays < 0:
            raise AcnError("ExpertParallelRenderer: tile_rays must be >= 0")
        self.own, self.eo = own, eo
        self.split_send = [e * Cc for e in eo]
        self.split_recv = [E * Cc] * W
        self.split_cnt_send, self.split_cnt_recv = list(eo), [E] * W
        dev = model.submodules[0].xyz_encoder.hash_table.device
        self.device = dev
        f32 = dict(device=dev, dtype=torch.float32)
        i32 = dict(device=dev, dtype=torch.int32)
        L = _lib.lib()
        self.rays = torch.zeros(N, 8, **f32)
        self.t = torch.empty(N, S, **f32)
        self.seg = torch.zeros(2 * K + 1, device=dev, dtype=torch.int64)
        self.rws = torch.empty(int(L.acn_routed_workspace_bytes(M, K)), device=dev, dtype=torch.uint8)
        self.pidx = torch.empty(K * Cc, **i32)
        self.pw = torch.empty(K * Cc, **f32)
        self.pk = torch.empty(K * Cc, **i32)
        self.xd = torch.zeros(K * Cc, 6, **f32)
        self.pmap = torch.empty(M, K, **i32)
        self.yr = torch.zeros(K * Cc, 4, **f32)
        R = W * E * Cc
        self.recv_cnt = torch.zeros(W * E, device=dev, dtype=torch.int64)
        self.recv_xd = torch.zeros(R, 6, **f32)
        self.ret = torch.zeros(R, 4, **f32)
        self.rgb = torch.empty(N, 3, **f32)
        self.depth = torch.empty(N, **f32)
        self.acc = torch.empty(N, **f32)
        self.weights = torch.empty(N, S, **f32) if want_weights else None
        self.routing = model.routing_spec()
        self.hard = 0 if self.routing.boundary_margin > 1.0 else 1
        with torch.no_grad():   # an inference renderer: the head's spec, whatever the caller's grad mode
            self.bg = _fused_background(model, bg_color_default, N, dev)
        if self.bg is None:
            raise AcnError(f"ExpertParallelRenderer: background policy {bg_color_default!r} needs the composed path")
        self.bg_spec, self._bg_keep = self.bg if isinstance(self.bg, tuple) else (self.bg, None)
        # the owned experts' packed images (acn_pack_experts with a routing of K = E): packed per call from the
        # live parameters, so a captured call renders the current weights
        self.own_specs = [model.submodules[k].expert_spec(None) for k in own]
        self.own_routing = ops.make_routing(torch.zeros(E, 3), E, True, 1.0)
        self.packed = torch.empty(E * int(L.acn_workspace_bytes(1)) // 4, **f32)
        self._own_arr = ops._experts_array(self.own_specs)
        self.graph = None
        self._graph_wanted = bool(graph)
        self.replays = 0
        self.owner = owner
        _GRAPH_OWNERS.add(self)
        self.last_exchange = None    # bytes this rank sent in the last call: {"sent": .., "live": ..}

    def _run(self, n: int) -> None:
        import ctypes as C
        from . import _lib, ops
        from ._lib import check, ptr
        L = _lib.lib()
        s = int(torch.cuda.current_stream(self.device).cuda_stream)
        K, E, S, Cc, comm = self.K, self.E, self.S, self.C, self.comm
        caps = (C.c_int64 * K)(*([Cc] * K))
        check(L.acn_routed_count_caps_tiled(ptr(self.rays), n, S, None, C.byref(self.routing), caps, self.tile_rays,
                                            ptr(self.t), ptr(self.seg), ptr(self.rws), self.rws.numel(), s),
              "acn_routed_count_caps_tiled")
        check(L.acn_routed_scatter_xd_tiled(ptr(self.rays), n, S, K, self.tile_rays, ptr(self.t), ptr(self.seg),
                                            ptr(self.rws), ptr(self.pidx), ptr(self.pw), ptr(self.xd), ptr(self.pmap),
                                            ptr(self.pk), s), "acn_routed_scatter_xd_tiled")
        comm.all_to_all(self.recv_cnt, self.seg[K + 1:], self.split_cnt_recv, self.split_cnt_send)
        comm.all_to_all(self.recv_xd, self.xd, self.split_recv, self.split_send)
        check(L.acn_pack_experts(self._own_arr, C.byref(self.own_routing), -1, ptr(self.packed),
                                 self.packed.numel() * 4, s), "acn_pack_experts")
        hook = ops.EVENT_HOOK if not torch.cuda.is_current_stream_capturing() else None   # bench.py timing
        if hook is not None:
            e0 = torch.cuda.Event(enable_timing=True)
            e0.record()
        check(L.acn_ep_field_fwd(ptr(self.recv_xd), ptr(self.recv_cnt), self.W, E, Cc, self._own_arr,
                                 ptr(self.packed), self.packed.numel() * 4, ptr(self.ret), s), "acn_ep_field_fwd")
        if hook is not None:
            e1 = torch.cuda.Event(enable_timing=True)
            e1.record()
            hook.append((e0, e1))
        comm.all_to_all(self.yr, self.ret, self.split_send, self.split_recv)
        check(L.acn_ep_composite(ptr(self.rays), n, S, None, ptr(self.yr), ptr(self.pw), ptr(self.pmap), K, self.hard,
                                 C.byref(self.bg_spec), 1.0, 0.0, ptr(self.rgb), ptr(self.depth), ptr(self.weights),
                                 ptr(self.acc), s), "acn_ep_composite")

    def _run_planned(self, n: int, counts, recv_cnt: Tensor, pack: bool = True) -> None:
        """One batch with the exchange sized by ``counts`` (host (W, K) ints: every rank's pair counts of this
        batch, the capacities of its segments): compact layouts on both sides, no padding slot crosses a link.
        ``recv_cnt``: the (W, E) counts of the owned experts on the device (int64; read by the field kernel)."""
        import ctypes as C
        from . import _lib
        from ._lib import check, ptr
        L = _lib.lib()
        s = int(torch.cuda.current_stream(self.device).cuda_stream)
        K, E, W, S, comm, rank, own, owner = self.K, self.E, self.W, self.S, self.comm, self.comm.rank, self.own, self.owner
        mine = [int(c) for c in counts[rank]]
        caps = (C.c_int64 * K)(*mine)
        check(L.acn_routed_count_caps_tiled(ptr(self.rays), n, S, None, C.byref(self.routing), caps, self.tile_rays,
                                            ptr(self.t), ptr(self.seg), ptr(self.rws), self.rws.numel(), s),
              "acn_routed_count_caps_tiled")
        check(L.acn_routed_scatter_xd_tiled(ptr(self.rays), n, S, K, self.tile_rays, ptr(self.t), ptr(self.seg),
                                            ptr(self.rws), ptr(self.pidx), ptr(self.pw), ptr(self.xd), ptr(self.pmap),
                                            ptr(self.pk), s), "acn_routed_scatter_xd_tiled")
        send = [sum(mine[k] for k in range(K) if owner[k] == o) for o in range(W)]
        rc = [int(counts[w][k]) for w in range(W) for k in own]
        recv = [sum(rc[w * E:(w + 1) * E]) for w in range(W)]
        ps, pr = sum(send), sum(recv)
        comm.all_to_all(self.recv_xd[:pr], self.xd[:ps], recv, send)
        if pack:   # the owned experts' images: constant within a frame, packed by its first batch
            check(L.acn_pack_experts(self._own_arr, C.byref(self.own_routing), -1, ptr(self.packed),
                                     self.packed.numel() * 4, s), "acn_pack_experts")
        if pr > 0:
            from . import ops
            hook = ops.EVENT_HOOK   # bench.py timing (eager only: this path is never captured)
            if hook is not None:
                e0 = torch.cuda.Event(enable_timing=True)
                e0.record()
            check(L.acn_ep_field_fwd_compact(ptr(self.recv_xd), ptr(recv_cnt), W, E, 0, max(rc), self._own_arr,
                                             ptr(self.packed), self.packed.numel() * 4, ptr(self.ret), s),
                  "acn_ep_field_fwd_compact")
            if hook is not None:
                e1 = torch.cuda.Event(enable_timing=True)
                e1.record()
                hook.append((e0, e1))
        comm.all_to_all(self.yr[:ps], self.ret[:pr], send, recv)
        check(L.acn_ep_composite(ptr(self.rays), n, S, None, ptr(self.yr), ptr(self.pw), ptr(self.pmap), K, self.hard,
                                 C.byref(self.bg_spec), 1.0, 0.0, ptr(self.rgb), ptr(self.depth), ptr(self.weights),
                                 ptr(self.acc), s), "acn_ep_composite")
        # sent: the records out (24 B) and the results of the received records back (16 B); the live pairs of this
        # rank are ps (its records) and pr (the records it evaluates for the others)
        self.last_exchange = {"sent": 24 * ps + 16 * pr, "live": 24 * ps + 16 * pr, "pairs_sent": ps,
                              "pairs_evaluated": pr}

    def render_planned(self, rays: Tensor, counts, recv_cnt: Optional[Tensor] = None, pack: bool = True):
        """As __call__, with the exchange sized by ``counts`` (host (W, K): every rank's pair counts of this batch,
        acn_routed_count_batches).  Eager (the split sizes change per batch); collective over the group.
        ``recv_cnt``: counts[w][own[e]] as a device int64 (W * E) tensor, if the caller already holds one."""
        from ._lib import AcnError
        n = int(rays.shape[0])
        if rays.dim() != 2 or rays.shape[1] != 8 or not 0 < n <= self.N:
            raise AcnError(f"ExpertParallelRenderer was built for up to {self.N} rays per rank; got {tuple(rays.shape)}")
        self.rays[:n].copy_(rays, non_blocking=True)
        if recv_cnt is None:   # a fresh device tensor per call: a reused pinned buffer could be rewritten before
            recv_cnt = torch.tensor([int(counts[w][k]) for w in range(self.W) for k in self.own],   # its copy ran
                                    dtype=torch.int64).to(self.device)
        self._run_planned(n, counts, recv_cnt, pack)
        w = self.weights[:n] if self.weights is not None else None
        return self.rgb[:n], self.depth[:n], w, self.acc[:n]

    def __call__(self, rays: Tensor):
        """(rgb (n,3), depth (n,), weights (n,S) or None, acc (n,)) of this rank's ``rays`` (n <= n_rays): views
        of persistent buffers, valid until the next call.  Collective over the group."""
        from ._lib import AcnError
        n = int(rays.shape[0])
        if rays.dim() != 2 or rays.shape[1] != 8 or not 0 < n <= self.N:
            raise AcnError(f"ExpertParallelRenderer was built for up to {self.N} rays per rank; got {tuple(rays.shape)}")
        self.rays[:n].copy_(rays, non_blocking=True)
        self.last_exchange = {"sent": 8 * self.K + (24 + 16) * sum(self.split_send), "live": None}
        if n == self.N and self.graph is not None:
            self.graph.replay()
            self.replays += 1
        else:
            self._run(n)
            if n == self.N and self._graph_wanted and self.graph is None:
                torch.cuda.synchronize(self.device)
                g = torch.cuda.CUDAGraph()
                with graph_capture(g):
                    self._run(self.N)
                torch.cuda.synchronize(self.device)
                self.graph = g
        w = self.weights[:n] if self.weights is not None else None
        return self.rgb[:n], self.depth[:n], w, self.acc[:n]

    def close(self) -> int:
        """Destroy the captured graph (its RCCL resources go with it); the next full call captures again.
        Returns 1 when a graph was released."""
        if self.graph is None:
            return 0
        torch.cuda.synchronize(self.device)
        self.graph.reset()
        self.graph = None
        return 1

    def overflowed(self) -> bool:
        """True when the last call's pairs of some expert exceeded the capacity (host read of the counts)."""
        return bool(int(self.seg[self.K + 1: 2 * self.K + 1].max()) > self.C)


def _renderer_for(model, n: int, S: int, group, cap: Optional[int]) -> ExpertParallelRenderer:
    """The ExpertParallelRenderer cached on ``model`` for (batch, samples, group, capacity)."""
    cache = model.__dict__.setdefault("_acn_ep_renderers", {})
    key = (n, S, id(group), cap)
    r = cache.get(key)
    if r is None:
        r = cache[key] = ExpertParallelRenderer(model, n, S, group=group, capacity=cap)
    return r


@torch.no_grad()
def render_rays_ep_batched(model, rays: Tensor, ray_samples: int, group=None, batch: int = 32768,
                           capacity_frac: Optional[float] = None, stats: Optional[dict] = None):
    """(rgb, depth, acc) of this rank's ``rays`` through ExpertParallelRenderer in batches of ``batch`` rays.
    Every rank must make the same number of calls: the batch count is agreed on with one all-reduce (MAX) of
    the rank's batch count.

    Default (``capacity_frac`` None): the planned exchange.  One routing pass over the rank's rays counts the
    pairs of every (batch, expert) (acn_routed_count_batches), one all-gather gives every rank all counts and
    ONE host read per frame sizes every batch's all-to-alls to exactly its live pairs (40 B each: the 24-B
    record out, the 16-B (rgb, sigma) back); the counts each batch actually routed are checked against the
    plan at the end (the same routing arithmetic: a mismatch raises).
    ``capacity_frac`` in (0, 1]: the fixed layout of ExpertParallelRenderer -- every (sender, expert) segment
    holds that share of a batch's samples; the counts of all batches are read back once at the end and any
    overflowed batch is re-rendered at full capacity (collectively).
    ``stats``: filled with the bytes this rank sent ("sent") and the live pair bytes ("live") over the frame."""
    world, rank = world_rank(group)
    n, S = int(rays.shape[0]), int(ray_samples)
    dev = rays.device
    nb = (n + batch - 1) // batch
    if world > 1:
        t = torch.tensor([nb], dtype=torch.int64, device=dev)
        _Comm(group).all_reduce_max(t)
        nb = int(t)
    if capacity_frac is None:
        return _render_planned(model, rays, S, group, batch, nb, stats)
    M = batch * S
    cap = None if capacity_frac >= 1.0 else max(1, int(M * capacity_frac))
    r = _renderer_for(model, batch, S, group, cap)
    rgb = torch.empty(n, 3, device=dev)
    depth = torch.empty(n, device=dev)
    acc = torch.empty(n, device=dev)
    K = r.K
    counts = torch.zeros(nb, K, device=dev, dtype=torch.int64)
    dummy = rays[:1] if n else torch.zeros(1, 8, device=dev)
    for b in range(nb):
        lo, hi = b * batch, min(n, (b + 1) * batch)
        sub = rays[lo:hi] if hi > lo else dummy       # a rank with fewer rays still joins the collectives
        o = r(sub)
        if hi > lo:
            rgb[lo:hi], depth[lo:hi], acc[lo:hi] = o[0], o[1], o[3]
        counts[b] = r.seg[K + 1: 2 * K + 1]
    if cap is not None:
        over = (counts.max(dim=1).values > cap).to(torch.int64)
        if world > 1:
            _Comm(group).all_reduce_max(over)
        redo = [b for b in range(nb) if int(over[b])]       # the one host read of the frame
        if redo:
            full = _renderer_for(model, batch, S, group, None)
            for b in redo:
                lo, hi = b * batch, min(n, (b + 1) * batch)
                o = full(rays[lo:hi] if hi > lo else dummy)
                if hi > lo:
                    rgb[lo:hi], depth[lo:hi], acc[lo:hi] = o[0], o[1], o[3]
    return rgb, depth, acc


def _render_planned(model, rays: Tensor, S: int, group, batch: int, nb: int, stats: Optional[dict]):
    """render_rays_ep_batched's planned exchange (see there)."""
    import ctypes as C
    from . import _lib
    from ._lib import AcnError, check, ptr
    world, rank = world_rank(group)
    n = int(rays.shape[0])
    dev = rays.device
    r = _renderer_for(model, batch, S, group, None)
    K = r.K
    L = _lib.lib()
    plan = torch.zeros(nb, K, device=dev, dtype=torch.int64)
    s = int(torch.cuda.current_stream(dev).cuda_stream)
    if n:
        check(L.acn_routed_count_batches(ptr(rays.contiguous()), n, S, batch, None, C.byref(r.routing), ptr(plan), s),
              "acn_routed_count_batches")
    if r.comm.direct:
        allp = torch.empty(world * nb, K, device=dev, dtype=torch.int64)
        if r.comm.staged:
            parts = [torch.empty(nb, K, dtype=torch.int64) for _ in range(world)]
            dist.all_gather(parts, plan.cpu(), group=group)
            allp = torch.cat(parts)
        else:
            dist.all_gather_into_tensor(allp, plan, group=group)
        host = allp.view(world, nb, K).cpu().tolist()      # the one host read of the frame's plan
    else:
        host = [plan.cpu().tolist()]
    rgb = torch.empty(n, 3, device=dev)
    depth = torch.empty(n, device=dev)
    acc = torch.empty(n, device=dev)
    seen = torch.zeros(nb, K, device=dev, dtype=torch.int64)
    dummy = rays[:1] if n else torch.zeros(1, 8, device=dev)
    # every batch's received counts of the owned experts, on the device in one copy
    rc_all = torch.tensor([[host[w][b][k] for w in range(world) for k in r.own] for b in range(nb)],
                          dtype=torch.int64).to(dev)
    sent = evaluated = 0
    for b in range(nb):
        lo, hi = b * batch, min(n, (b + 1) * batch)
        counts = [host[w][b] for w in range(world)]
        o = r.render_planned(rays[lo:hi] if hi > lo else dummy, counts, rc_all[b], pack=b == 0)
        if hi > lo:
            rgb[lo:hi], depth[lo:hi], acc[lo:hi] = o[0], o[1], o[3]
            seen[b] = r.seg[K + 1: 2 * K + 1]
        sent += r.last_exchange["sent"]
        evaluated += r.last_exchange["pairs_evaluated"]
    if n and not torch.equal(seen[: (n + batch - 1) // batch], plan[: (n + batch - 1) // batch]):
        raise AcnError("render_rays_ep_batched: a batch routed other pair counts than its plan")
    if stats is not None:
        # live: 24 B per pair this rank's rays actually routed (the device counts of every batch, independent of
        # the split sizes the exchange used) + 16 B per pair it evaluated for the senders (their own plans, which
        # each sender checks against its routed counts the same way)
        stats.update(sent=sent, live=24 * int(seen.sum()) + 16 * evaluated, batches=nb)
    return rgb, depth, acc


@torch.no_grad()
def render_image_expert_parallel(model, *, H: int, W: int, fx: float, fy: float, cx: float, cy: float, c2w: Tensor,
                                 scene_box, ray_samples: int = 64, center_pixels: bool = True,
                                 gt_srgb: Optional[Tensor] = None, metrics_space: str = "linear", group=None,
                                 backend=None, rays: Optional[Tensor] = None, batch: int = 32768,
                                 capacity_frac: Optional[float] = None, stats: Optional[dict] = None):
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
    plan = contiguous_plan(rays.shape[0], world, rays.device)
    idx = plan.indices(rank).to(rays.device)
    if backend is not None:   # a compute backend (tests: the CPU restatement) through the eager exchange
        rgb, depth, _, acc = render_rays_expert_parallel(backend, rays[idx].contiguous(), ray_samples,
                                                         len(model.submodules), group)
    else:
        rgb, depth, acc = render_rays_ep_batched(model, rays[idx].contiguous(), ray_samples, group=group,
                                                 batch=batch, capacity_frac=capacity_frac, stats=stats)
    local = torch.cat([rgb.float().view(-1, 3), depth.float().view(-1, 1), acc.float().view(-1, 1)], dim=1)
    full = gather_rendered(local, plan, group)
    rgb_img = full[:, :3].reshape(H, W, 3).clamp_(0, 1)
    psnr = None
    if gt_srgb is not None:
        sse, cnt = local_sse(rgb_img.view(-1, 3)[idx], gt_srgb.to(rgb_img.device).view(-1, 3)[idx], metrics_space)
        psnr = psnr_reduce(sse, cnt, rgb_img.device, group)
    return rgb_img, full[:, 3], full[:, 4], psnr


# ============================================================================ sync-free expert-parallel step
FORCE_COLLECTIVES = False   # tests: the exchanges through the process group even at world size 1 (RCCL on one GPU)

# Owners of HIP graphs that captured collectives (ExpertParallelRenderer / ExpertParallelAdaptStep).  RCCL ties a
# communicator's resources to every graph that captured one of its collectives and releases them only when that
# graph is destroyed; ncclCommDestroy waits for them, so destroy_process_group() (and the interpreter's exit
# handlers that run it) never return while such a graph is alive.  shutdown() releases them first.
import weakref as _weakref
_GRAPH_OWNERS = _weakref.WeakSet()


def release_collective_graphs() -> int:
    """Destroy every live graph held by an ExpertParallelRenderer / ExpertParallelAdaptStep (they recapture on
    their next full call).  Returns how many were released."""
    n = 0
    for o in list(_GRAPH_OWNERS):
        n += o.close()
    return n


def shutdown(group=None, timeout: float = 120.0) -> bool:
    """Release the collective-capturing graphs, synchronize, then destroy_process_group(group) -- bounded: a
    teardown that does not return within ``timeout`` seconds is reported (False) instead of hanging the caller.
    Reference: the process group's lifetime in scripts/create_clusters.py:224-238."""
    import gc
    import threading
    release_collective_graphs()
    gc.collect()
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    done = threading.Event()

    def _destroy():
        dist.destroy_process_group(group)
        done.set()
    t = threading.Thread(target=_destroy, daemon=True, name="acn-pg-teardown")
    t.start()
    t.join(timeout)
    return done.is_set()



class _Comm:
    """The step's collectives on device buffers of host-known constant sizes (no count exchange on the
    host): RCCL directly (``nccl`` backend), ``gloo`` through staged host copies (the multi-process tests of
    this same exchange code on one GPU or on CPU-only hosts), plain copies at world size 1."""

    def __init__(self, group=None):
        self.world, self.rank = world_rank(group)
        self.group = group
        # FORCE_COLLECTIVES: run the collectives even at world size 1 (tests: RCCL on one GPU)
        self.force = FORCE_COLLECTIVES and dist.is_available() and dist.is_initialized()
        self.direct = self.world > 1 or self.force
        self.staged = self.direct and dist.get_backend(group) == "gloo"

    def all_to_all(self, out: Tensor, inp: Tensor, out_splits: Sequence[int], in_splits: Sequence[int]) -> None:
        if not self.direct:
            out.copy_(inp)
        elif self.staged:
            oc = torch.empty(out.shape, dtype=out.dtype)
            dist.all_to_all_single(oc, inp.cpu(), list(out_splits), list(in_splits), group=self.group)
            out.copy_(oc)
        else:
            dist.all_to_all_single(out, inp, list(out_splits), list(in_splits), group=self.group)

    def all_reduce(self, t: Tensor) -> None:
        if not self.direct:
            return
        if self.staged:
            c = t.cpu()
            dist.all_reduce(c, group=self.group)
            t.copy_(c)
        else:
            dist.all_reduce(t, group=self.group)

    def all_reduce_max(self, t: Tensor) -> None:
        if not self.direct:
            return
        if self.staged:
            c = t.cpu()
            dist.all_reduce(c, op=dist.ReduceOp.MAX, group=self.group)
            t.copy_(c)
        else:
            dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.group)


class ExpertParallelAdaptStep:
    """runtime_adapt's update of the routed container (runtime_adapt.py:286-309, active_module None) with
    the experts distributed over the ranks of ``group`` -- expert k on rank expert_owner(K, W)[k] -- and no
    host synchronisation: every exchange has a constant size, so a step is a fixed sequence of launches and
    collectives that a HIP graph can hold (at world size 1 the exchanges are copies and ``graph=True``
    captures the step after ``warmup`` eager real steps; at W > 1 the RCCL collectives run eagerly by default,
    ``graph=True`` opts in to capturing them as well).

    Per step, on every rank:
      sender  rays (this rank's shard) -> t, routing, (sample, expert) pairs in the FIXED layout of
              acn_routed_count_fixed (expert k at [k C, (k+1) C), C = n_rays * S >= any expert's count) as
              24-B xd records -- grouped by owner, so the pair buffer is the all-to-all send buffer
      a2a #0  the per-expert live counts (int64) to the owners;  a2a #1 the xd records (constant splits)
      owner   acn_ep_gather: compact per-expert pair lists (padded to 128) -> hash grid + fused MLP of its
              experts -> acn_ep_scatter_back into the received layout
      a2a #2  (rgb, sigma) back to the senders, at their pairs' slots -> blend (expert order) + background +
              compositing + loss (scaled by n / N_global: the global mean)
      a2a #3  dL/d(rgb, sigma) back to the owners -> fused MLP backward + table scatter of the owned experts;
              the background head's gradients all-reduced (sum over the ranks' rays)
      update  optim.SlottedAdam over the owned experts (an expert no rank routed a sample to is skipped, as
              torch skips grad None) + the replicated head; clip norm = all-reduced owned part + the head once.
    ``n_rays_global``: the batch the loss averages over -- W * n (weak: every rank streams its own batches) or
    the reference's batch split over the ranks (strong: each rank holds n = N / W of one runtime_adapt batch,
    and the update is exactly that batch's).  Reference: models/inr/meta_container.py:300-337."""

    def __init__(self, P, model, n_rays: int, optimizer: FusedAdam, n_rays_global: Optional[int] = None,
                 grad_clip: Optional[float] = 1.0, group=None, graph: bool = False, warmup: int = 1,
                 jitter: str = "draw", clear_in_adam: bool = True, max_steps: int = 1 << 16,
                 capacity: Optional[int] = None):
        import ctypes as C
        import numpy as np
        from . import _lib, ops
        from ._lib import AcnError, acn_mlp
        from .meta_container import MetaContainer
        from .optim import NORM_ELSEWHERE_FLAG, ZERO_GRAD_FLAG, FusedAdam, SlottedAdam
        from .routed_train import ALIGN, FUSED_BACKGROUND, TELESCOPED_TABLE_NORM
        if not isinstance(model, MetaContainer) or not all(s._fusable for s in model.submodules):
            raise AcnError("ExpertParallelAdaptStep: a MetaContainer of reference-configuration experts is required")
        if not isinstance(optimizer, FusedAdam):
            raise AcnError("ExpertParallelAdaptStep needs FusedAdam")
        if not model.use_bg_nerf:
            raise AcnError("ExpertParallelAdaptStep: the background head is part of the reference configuration")
        encs = [s.xyz_encoder for s in model.submodules]
        e0 = encs[0]
        if any(e._res_host != e0._res_host or e.log2_hashmap_size != e0.log2_hashmap_size
               or e._interp_code != e0._interp_code for e in encs) or e0._interp_code == 0:
            raise AcnError("ExpertParallelAdaptStep: experts must share one Linear/Smoothstep hash-grid configuration")
        self.comm = comm = _Comm(group)
        W, rank = comm.world, comm.rank
        self.P, self.model, self.opt, self.grad_clip = P, model, optimizer, grad_clip
        self.mlp_precision = ops.TRAIN_MLP_PRECISION   # training MLP kernels (ops.set_train_mlp_precision)
        if self.mlp_precision == "amp":
            # the fp16 (use_amp) kernels need a loss scale, and this step carries none: gradients of
            # magnitude < 2^-24 would flush to zero (test_amp_underflow_without_loss_scale)
            raise AcnError("ExpertParallelAdaptStep: the use_amp MLP precision needs a loss scale this step does not "
                           "carry; select 'fp16x3' or 'fp32' (ops.set_train_mlp_precision)")
        self.jitter_mode = jitter
        self.clear_in_adam = bool(clear_in_adam)
        self.tele = TELESCOPED_TABLE_NORM and grad_clip is not None
        dev = e0.hash_table.device
        self.device = dev
        K = len(model.submodules)
        owner = expert_owner(K, W)
        own = [k for k in range(K) if owner[k] == rank]
        if not own:
            raise AcnError(f"ExpertParallelAdaptStep: rank {rank} owns no expert (K = {K} < W = {W})")
        E = len(own)
        eo = [owner.count(o) for o in range(W)]      # experts per owner (contiguous blocks)
        S, N = int(P.ray_samples), int(n_rays)
        M = N * S
        # capacity of one (sender, expert) segment of the exchange: M (never overflows) or smaller, sized to the
        # live records -- then a step whose pairs overflow on any rank is gated off on the device (zero upstream
        # gradients, no slot active in Adam: no update, no step count) and re-run at full capacity at the next
        # call (one small host read of the flag per step)
        # capacity="adaptive": full capacity for the warm-up steps, then per expert ~1.5x the largest count any rank
        # routed to it (all-reduced), regrown after an overflow (the graph is then captured again)
        self.adaptive = capacity == "adaptive"
        Cc = M if capacity is None or self.adaptive else max(1, min(M, int(capacity)))
        self.K, self.E, self.W, self.N, self.S, self.M, self.C = K, E, W, N, S, M, Cc
        self.own, self.eo = own, eo
        self.n_global = int(n_rays_global) if n_rays_global is not None else N * W
        self.split_cnt_send, self.split_cnt_recv = list(eo), [E] * W
        self.overflows = 0
        self.recaptures = 0
        self._check = None     # (event, n) of the last capacity-bounded step
        self.caps_dev = torch.full((K,), Cc, device=dev, dtype=torch.int64)
        self._set_caps([Cc] * K)
        Cc = M                 # buffers: full capacity (the re-run layout); a bounded layout uses their prefix
        f32 = dict(device=dev, dtype=torch.float32)
        i32 = dict(device=dev, dtype=torch.int32)
        i64 = dict(device=dev, dtype=torch.int64)
        L = _lib.lib()
        # ---- sender buffers
        self.rays = torch.zeros(N, 8, **f32)
        self.rgbs = torch.zeros(N, 3, **f32)
        self.u = torch.zeros(N, S, **f32)
        self.t = torch.empty(N, S, **f32)
        self.seg = torch.zeros(2 * K + 1, **i64)
        self.rws = torch.empty(int(L.acn_routed_workspace_bytes(M, K)), device=dev, dtype=torch.uint8)
        self.pidx = torch.empty(K * Cc, **i32)
        self.pw = torch.empty(K * Cc, **f32)
        self.pk = torch.empty(K * Cc, **i32)
        self.xd = torch.empty(K * Cc, 6, **f32)
        self.pmap = torch.empty(M, K, **i32)
        self.yr = torch.empty(K * Cc, 4, **f32)         # (rgb, sigma) of this rank's pairs, from the owners
        self.rgbs_dirs = torch.zeros(N, 3, **f32)
        # ---- owner buffers
        R = W * E * Cc                                   # received records
        cap = R + E * ALIGN                              # compact slots (segments padded to ALIGN)
        self.recv_cnt = torch.zeros(W * E, **i64)
        self.recv_xd = torch.empty(R, 6, **f32)
        self.eseg = torch.zeros(2 * E + 1, **i64)
        self.ews = torch.empty(int(L.acn_ep_workspace_bytes(W, E)), device=dev, dtype=torch.uint8)
        self.x01 = torch.empty(cap, 3, **f32)
        self.sh = torch.empty(cap, 16, **f32)
        self.pkl = torch.empty(cap, **i32)
        self.pflag = torch.empty(cap, **i32)
        self.back = torch.empty(cap, **i64)
        self.h0 = torch.empty(cap, 32, **f32)
        self.out = torch.empty(cap, 4, **f32)
        self.gh0 = torch.empty(cap, 32, **f32)
        self.gout = torch.empty(cap, 4, **f32)
        self.ret = torch.zeros(R, 4, **f32)
        self.recv_gy = torch.empty(R, 4, **f32)
        self.mws = torch.empty(int(ops.mlp_fn("acn_mlp_pairs_workspace_bytes", self.mlp_precision)(E)), device=dev,
                               dtype=torch.uint8)
        self.dw = torch.zeros(E, ops.MLP_DW_FLOATS, **f32)
        self.loss = torch.zeros((), **f32)
        self.loss_global = torch.zeros(1, **f32)
        self.ovf = torch.zeros(1, **i64)                # global overflow flag of the last step (device)
        self.ovf_host = torch.zeros(1, dtype=torch.int64, pin_memory=True)
        self.keep = torch.ones((), **f32)               # 1 - overflow: gates the upstream gradients
        self.ovf_b = torch.zeros(1, device=dev, dtype=torch.bool)
        # ---- persistent gradients of the owned experts and the (replicated) background head
        self.gtables = [torch.zeros_like(encs[k].hash_table) for k in own]
        self.bg_params = list(model.bg_mlp.parameters())
        nbg = sum(p.numel() for p in self.bg_params)
        self.gbg_flat = torch.zeros(nbg, **f32)
        self.gbg, o = [], 0
        for p in self.bg_params:
            self.gbg.append(self.gbg_flat[o:o + p.numel()].view_as(p))
            o += p.numel()
        try:
            self.bg_spec, self._bg_keep = model.background_spec() if FUSED_BACKGROUND else (None, None)
        except AcnError:
            self.bg_spec, self._bg_keep = None, None
        slot_of, zero_of = {}, set()
        for j, k in enumerate(own):
            sub = model.submodules[k]
            sub.xyz_encoder.hash_table.grad = self.gtables[j]
            slot_of[id(sub.xyz_encoder.hash_table)] = j
            zero_of.add(id(sub.xyz_encoder.hash_table))
            views, off = [], 0
            for shp in ops.MLP_DW_SHAPES:
                n = int(np.prod(shp))
                views.append(self.dw[j, off:off + n].view(shp))
                off += n
            for (name, t), g in zip(sub._mlp_tensors(None).items(), views):
                t.grad = g
                slot_of[id(t)] = j
        for p, g in zip(self.bg_params, self.gbg):
            p.grad = g
            slot_of[id(p)] = E
        self._mlp_structs = [ops._mlp_struct([t for t in model.submodules[k]._mlp_tensors(None).values()]) for k in own]
        self._mlp_ptrs = (C.POINTER(acn_mlp) * E)(*[C.pointer(w) for w in self._mlp_structs])
        self._tables = (C.c_void_p * E)(*[encs[k].hash_table.data_ptr() for k in own])
        self._gtables = (C.c_void_p * E)(*[g.data_ptr() for g in self.gtables])
        self._res = (C.c_int32 * len(e0._res_host))(*e0._res_host)
        boxes = [model.submodules[k]._host_box() for k in own]
        self._mins = (C.c_float * (3 * E))(*[float(v) for b in boxes for v in b[0]])
        self._exts = (C.c_float * (3 * E))(*[float(v) for b in boxes for v in b[1]])
        lo = np.float32(1e-6)
        self._lo, self._hi = C.c_float(lo), C.c_float(np.float32(1.0) - lo)
        self.routing = model.routing_spec()
        grads = {i: None for i in slot_of}
        for p in model.parameters():
            if id(p) in slot_of:
                grads[id(p)] = p.grad
        flags = {i: (ZERO_GRAD_FLAG if self.clear_in_adam else 0) | (NORM_ELSEWHERE_FLAG if self.tele else 0)
                 for i in zero_of}
        self.adam = SlottedAdam(optimizer, slot_of, grads, E, E + 1, flags, max_steps=max_steps, split_norm=W > 1)
        self.table_sumsq = torch.zeros(1, device=dev, dtype=torch.float64)
        self._params = [r[0] for r in self.adam.rows]
        self.replays = 0
        self.steps_done = 0
        self.graph = None
        self._eager_left = max(1, int(warmup)) if graph else 0
        _GRAPH_OWNERS.add(self)

    def _set_caps(self, caps) -> None:
        """Per-expert segment capacities (identical on every rank) and the layouts / split sizes they imply."""
        import ctypes as C
        self.caps = [int(max(1, min(self.M, c))) for c in caps]
        self.caps_dev.copy_(torch.tensor(self.caps, dtype=torch.int64))
        self._caps_c = (C.c_int64 * self.K)(*self.caps)
        self._own_caps_c = (C.c_int64 * self.E)(*[self.caps[k] for k in self.own])
        owner = expert_owner(self.K, self.W)
        self.split_send = [sum(self.caps[k] for k in range(self.K) if owner[k] == o) for o in range(self.W)]
        self.split_recv = [sum(self.caps[k] for k in self.own)] * self.W
        self.slots_send, self.slots_recv = sum(self.split_send), sum(self.split_recv)
        self.bounded = any(c < self.M for c in self.caps)

    def exchange_bytes(self) -> int:
        """Bytes this rank sends per step over the four all-to-alls at the current capacities: the counts (8 B
        per expert), then per pair slot the record (24 B), the (rgb, sigma) result (16 B) and its gradient
        (16 B) -- the sends of this rank's records and results summed with those of its gradients."""
        return 8 * self.K + 24 * self.slots_send + 16 * self.slots_recv + 16 * self.slots_send

    def _step(self, n: int, full: bool = False) -> None:
        import ctypes as C
        from . import _lib, ops
        from ._lib import check, ptr
        from .ray_rendering import volume_render
        from .routed_train import ALIGN, JITTER
        from .train import mse_color_loss
        L = _lib.lib()
        saved = None
        if full and self.bounded:      # the full-capacity re-run of an overflowed step
            saved = list(self.caps)
            self._set_caps([self.M] * self.K)
        bounded = self.bounded
        Cc = self.C
        dev, K, E, S, comm = self.device, self.K, self.E, self.S, self.comm
        s = int(torch.cuda.current_stream(dev).cuda_stream)
        M = n * S
        if not self.clear_in_adam:
            for g in self.gtables:
                g.zero_()
        u, t = self.u[:n], self.t[:n]
        if self.jitter_mode == "draw":
            u.copy_(JITTER(n, S, dev))   # the reference's rand_like(low) draw
        # sender: pairs in the fixed owner-grouped layout
        check(L.acn_routed_count_caps(ptr(self.rays), n, S, ptr(u), C.byref(self.routing), self._caps_c, ptr(t),
                                      ptr(self.seg), ptr(self.rws), self.rws.numel(), s), "acn_routed_count_caps")
        check(L.acn_routed_scatter_xd(ptr(self.rays), n, S, K, ptr(t), ptr(self.seg), ptr(self.rws), ptr(self.pidx),
                                      ptr(self.pw), ptr(self.xd), ptr(self.pmap), ptr(self.pk), s),
              "acn_routed_scatter_xd")
        check(L.acn_routed_pad_pairs(ptr(self.seg), K, max(self.caps), ptr(self.pidx), ptr(self.pw), s),
              "acn_routed_pad_pairs")
        if bounded:   # any rank's expert past its capacity: the whole step is gated off (device flag, all-reduced)
            torch.any(torch.gt(self.seg[K + 1: 2 * K + 1], self.caps_dev), dim=0, keepdim=True, out=self.ovf_b)
            self.ovf.copy_(self.ovf_b)
            comm.all_reduce_max(self.ovf)
            self.keep.copy_(1.0 - self.ovf.to(torch.float32).view(()))
        comm.all_to_all(self.recv_cnt, self.seg[K + 1:], self.split_cnt_recv, self.split_cnt_send)
        comm.all_to_all(self.recv_xd[:self.slots_recv], self.xd[:self.slots_send], self.split_recv, self.split_send)
        # owner: compact pair lists of the owned experts, field, results back into the received layout
        check(L.acn_ep_gather_caps(ptr(self.recv_xd), ptr(self.recv_cnt), self.W, E, self._own_caps_c, ALIGN,
                              C.cast(self._mins, C.c_void_p), C.cast(self._exts, C.c_void_p), self._lo, self._hi,
                              ptr(self.eseg), ptr(self.ews), ptr(self.x01), ptr(self.sh), ptr(self.pkl),
                              ptr(self.pflag), ptr(self.back), s), "acn_ep_gather")
        enc = self.model.submodules[self.own[0]].xyz_encoder
        check(L.acn_hashgrid_fwd_pairs(ptr(self.x01), ptr(self.pkl), ptr(self.eseg), E, self._tables, self._res,
                                       len(enc._res_host), enc.log2_hashmap_size, enc._interp_code, ptr(self.h0), s),
              "acn_hashgrid_fwd_pairs")
        mfn = lambda name: ops.mlp_fn(name, self.mlp_precision)  # noqa: E731
        check(mfn("acn_mlp_pack_pairs")(self._mlp_ptrs, E, ptr(self.mws), s), "acn_mlp_pack_pairs")
        check(mfn("acn_mlp_train_fwd_pairs")(ptr(self.h0), ptr(self.sh), ptr(self.eseg), E, ptr(self.mws), ptr(self.out), s),
              "acn_mlp_train_fwd_pairs")
        check(L.acn_ep_scatter_back(ptr(self.out), ptr(self.back), ptr(self.eseg), E, ptr(self.ret), s),
              "acn_ep_scatter_back")
        comm.all_to_all(self.yr[:self.slots_send], self.ret[:self.slots_recv], self.split_send, self.split_recv)
        # sender: blend, background, compositing, loss (the global batch mean), their gradients
        rs = ops.routed_blend_fwd(self.yr, self.pw, self.pmap[:M]).view(n, S, 4).requires_grad_(True)
        rays, rgbs, dirs = self.rays[:n], self.rgbs[:n], self.rgbs_dirs[:n]
        # the loss averages over the global batch: a full batch is n_global / W rays per rank (weak) or the
        # configured share (strong); a ragged batch (n < n_rays, world size 1 only) averages over its own n rays
        frac = float(n) / float(self.n_global) if n == self.N else 1.0
        if self.bg_spec is not None:
            dirs.copy_(rays[:, 3:6])
            bg = ops.background_fwd(dirs, self.bg_spec).requires_grad_(True)
            with torch.enable_grad():
                rgb = volume_render(rs, t, bg_rgb=bg)[0]
                loss = mse_color_loss(rgb, rgbs, self.P.color_space) * frac
                g_rs, g_bg = torch.autograd.grad(loss, [rs, bg])
            if bounded:
                g_rs, g_bg = g_rs * self.keep, g_bg * self.keep
            ops.background_bwd(dirs, self.bg_spec, g_bg, self.gbg)
        else:
            with torch.enable_grad():
                bg = self.model.background_color(rays[:, 3:6])
                rgb = volume_render(rs, t, bg_rgb=bg)[0]
                loss = mse_color_loss(rgb, rgbs, self.P.color_space) * frac
                grads = torch.autograd.grad(loss, [rs] + self.bg_params)
            g_rs = grads[0] * self.keep if bounded else grads[0]
            for g, buf in zip(grads[1:], self.gbg):
                buf.copy_(g * self.keep if bounded else g)
        self.loss.copy_(loss.detach())
        comm.all_reduce(self.gbg_flat)
        gy = ops.routed_blend_bwd(g_rs.reshape(M, 4).contiguous(), self.pidx[:self.slots_send], self.pw[:self.slots_send])
        comm.all_to_all(self.recv_gy[:self.slots_recv], gy, self.split_recv, self.split_send)
        # owner: backward of the owned experts
        check(L.acn_ep_gather_grad(ptr(self.recv_gy), ptr(self.back), ptr(self.eseg), E, ptr(self.gout), s),
              "acn_ep_gather_grad")
        check(mfn("acn_mlp_train_bwd_dw_pairs")(ptr(self.h0), ptr(self.sh), ptr(self.out), ptr(self.gout), ptr(self.eseg), E,
                                           ptr(self.mws), ptr(self.dw), ptr(self.gh0), s), "acn_mlp_train_bwd_dw_pairs")
        check(L.acn_hashgrid_bwd_pairs_sumsq(ptr(self.x01), ptr(self.pkl), ptr(self.pflag), ptr(self.eseg), E,
                                             ptr(self.gh0), self._gtables, self._res, len(enc._res_host),
                                             enc.log2_hashmap_size, enc._interp_code,
                                             ptr(self.table_sumsq) if self.tele else None, s),
              "acn_hashgrid_bwd_pairs_sumsq")
        from . import routed_train as RT
        if bounded:   # an overflowed step activates no slot: no moment decay, no step count (seg[E] < 0)
            self.eseg[E:E + 1].copy_(torch.where(self.ovf > 0, torch.full_like(self.ovf, -1), self.eseg[E:E + 1]))
        self.adam.step(self.eseg, self.grad_clip, self.table_sumsq if self.tele else None,
                       hook=RT.EVENT_HOOK if self.graph is None and not torch.cuda.is_current_stream_capturing()
                       else None,
                       allreduce=comm.all_reduce if self.W > 1 else None)   # the norm's split form: W > 1 only
        self.loss_global.copy_(self.loss.view(1))
        comm.all_reduce(self.loss_global)
        if saved is not None:
            self._set_caps(saved)

    def _adapt_caps(self, grow: float = 1.5) -> None:
        """Capacities from the last step's per-expert counts, all-reduced (MAX) so every rank agrees: ~grow x the
        largest count (at least 256 slots), never below the current capacity after a regrow; drops the graph
        (the split sizes changed) so the next full step is captured again."""
        c = self.seg[self.K + 1: 2 * self.K + 1].clone()
        self.comm.all_reduce_max(c)
        counts = [int(v) for v in c.cpu().tolist()]
        new = [max(256, int(grow * v) + 1) for v in counts]
        if grow > 1.5:
            new = [max(a, b) for a, b in zip(new, self.caps)]
        self._set_caps(new)
        if self.graph is not None:
            self._drop_graph()
            self._eager_left = 1
            self.recaptures += 1

    def _drop_graph(self) -> None:
        torch.cuda.synchronize(self.device)
        self.graph.reset()
        self.graph = None

    def close(self) -> int:
        """Settle the last step (flush), then destroy the captured graph and its RCCL resources; the next full
        step is captured again after one eager step.  Returns 1 when a graph was released."""
        self.flush()
        if self.graph is None:
            return 0
        self._drop_graph()
        self._eager_left = 1
        return 1

    def _capture(self) -> None:
        dev = self.device
        if self.adaptive and not self.bounded:
            self._adapt_caps()
        torch.cuda.synchronize(dev)
        g = torch.cuda.CUDAGraph()
        with graph_capture(g):
            self._step(self.N)
        torch.cuda.synchronize(dev)
        self.graph = g

    def __call__(self, rays: Tensor, rgbs: Tensor, jitter_u: Optional[Tensor] = None) -> Tensor:
        """One update on this rank's ``rays`` / ``rgbs`` (n <= n_rays); collective over the group.  Returns the
        global loss (device, 1 element)."""
        from ._lib import AcnError
        from .optim import bump_versions
        n = int(rays.shape[0])
        if rays.dim() != 2 or rays.shape[1] != 8 or tuple(rgbs.shape) != (n, 3) or not 0 < n <= self.N:
            raise AcnError(f"ExpertParallelAdaptStep was built for up to {self.N} rays per rank; got "
                           f"{tuple(rays.shape)}, {tuple(rgbs.shape)}")
        if self.adam.step0 + self.steps_done + 1 > self.adam.table_steps:
            raise AcnError("ExpertParallelAdaptStep: the Adam constant table is exhausted; build a new step object")
        if n != self.N and self.W > 1:
            # the global mean over a ragged global batch needs every rank's n: not known without a host exchange
            # on a path the ranks may not all take -- feed full batches (drop_last) at W > 1
            raise AcnError(f"ExpertParallelAdaptStep: ragged batch ({n} of {self.N} rays) at world size {self.W}; "
                           "use full batches (drop_last=True) with more than one rank")
        self.flush()    # the previous bounded step, re-run at full capacity if it overflowed
        self.rays[:n].copy_(rays, non_blocking=True)
        self.rgbs[:n].copy_(rgbs, non_blocking=True)
        if self.jitter_mode == "given":
            if jitter_u is None or tuple(jitter_u.shape) != (n, self.S):
                raise AcnError(f"ExpertParallelAdaptStep(jitter='given') needs jitter_u of shape ({n}, {self.S})")
            self.u[:n].copy_(jitter_u, non_blocking=True)
        if n == self.N and self.graph is not None:
            self.graph.replay()
            self.replays += 1
        else:
            self._step(n)
            if n == self.N and self._eager_left > 0:
                self._eager_left -= 1
                if self._eager_left == 0:
                    self._capture()
        if self.bounded:
            self.ovf_host.copy_(self.ovf, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record()
            self._check = (ev, n)
        self.steps_done += 1
        bump_versions(self._params)
        return self.loss_global

    def flush(self) -> None:
        """Settle the last capacity-bounded step: read its (global) overflow flag and, when set, redo that step
        at full capacity from the batch still in the static buffers (the overflowed attempt changed nothing).
        Called at the start of every step and by sync_state()."""
        if self._check is None:
            return
        ev, n = self._check
        self._check = None
        ev.synchronize()
        if int(self.ovf_host[0]):
            self.overflows += 1
            self._step(n, full=True)
            if self.adaptive:   # regrow from the true counts of the re-run, then capture again
                self._adapt_caps(grow=2.0)

    @property
    def last_norm(self) -> Tensor:
        return self.adam.scale

    def sync_state(self) -> None:
        """flush() + the host Adam state.  Call it at the end of an adaptation loop and before reading the
        parameters: a capacity-bounded step that overflowed is re-run only here or at the next call."""
        self.flush()
        self.adam.sync_state()

    def __del__(self):
        if getattr(self, "_check", None) is not None:
            import warnings
            warnings.warn("ExpertParallelAdaptStep dropped with an unsettled capacity-bounded step: call flush() "
                          "(or sync_state()) after the last step, or an overflowed last update is lost")
