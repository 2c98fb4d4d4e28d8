"""Online adaptation step (reference: pipelines/online_stage/runtime_adapt.py:213-315 ``runtime_adapt``,
nerfs/losses.py:10-32 ``compute_mse_loss``) on the HIP path.

One step = ``render_rays`` in training mode (stratified jitter) through the differentiable
per-expert forward -> sRGB/linear colour transform -> MSE -> backward (the hash-grid gather
backward is a HIP scatter-add kernel) -> ``clip_grad_norm_`` + Adam as one fused multi-tensor HIP
step (optim.FusedAdam).  The reference wraps the forward in fp16 autocast with a GradScaler; the default
fp16x3 MLP keeps fp32 accuracy, so no scale is needed; the use_amp precision (the reference's fp16
arithmetic, ops.set_train_mlp_precision("amp")) runs under a GradScaler like the reference's.

Expert-parallel use: ``adapt_step(..., group=)`` on the routed container
(active_module None, the online stage's call, runtime_adapt.py:88-90) distributes the experts over the
ranks of ``group`` (expert_parallel.py: all-to-all of per-sample records, complete per-expert
gradients on the owners, all-reduced background head, global clip norm): the update equals the
single-process one.  ``active_module=k`` adapts one expert with the container's background head; the
reference's own runtime_adapt cannot run that configuration (it renders ``base.submodules`` of the
expert itself), so it stays a single-process placement variant and refuses a group.
"""
from __future__ import annotations

import os
from typing import Dict, Iterable, Optional

import torch
import torch.nn.functional as F

from . import ops
from ._lib import graph_capture
from .color_space import color_space_transformer
from .optim import FusedAdam
from .ray_rendering import render_rays


class _MSELinearFn(torch.autograd.Function):
    """F.mse_loss(*color_space_transformer(pred, gt, 'linear')) as two HIP launches (loss.hip) instead of
    ~16 elementwise / reduction kernels; same float semantics (clamps pass NaN, powf, float scalars)."""

    @staticmethod
    def forward(ctx, pred, gt):
        ctx.save_for_backward(pred, gt)
        return ops.mse_linear_fwd(pred, gt)

    @staticmethod
    def backward(ctx, g):
        pred, gt = ctx.saved_tensors
        return ops.mse_linear_bwd(pred, gt, g.detach()), None


def mse_color_loss(pred_rgb, gt_rgb, color_space: str, reduction: str = "mean"):
    """F.mse_loss(*color_space_transformer(pred, gt, color_space)) (losses.py:10-32)."""
    from .ray_rendering import _second_order
    if (str(color_space).lower() == "linear" and reduction == "mean" and pred_rgb.is_cuda
            and pred_rgb.dtype == torch.float32 and pred_rgb.numel() > 0 and pred_rgb.shape == gt_rgb.shape
            and not _second_order()):
        return _MSELinearFn.apply(pred_rgb, gt_rgb.to(pred_rgb.device, torch.float32))
    pred_rgb, gt_rgb = color_space_transformer(pred_rgb, gt_rgb, color_space=color_space)
    return F.mse_loss(pred_rgb, gt_rgb, reduction=reduction)


def compute_mse_loss(P, model, data, params=None, active_module=None, reduction: str = "mean", **render_kwargs):
    """losses.py:10-32: MSE between render_rays(...) rgb and data['rgbs'] in P.color_space."""
    gt_rgb = data["rgbs"]
    rays = data["rays"]
    pred_rgb, *_ = render_rays(model, rays, ray_samples=P.ray_samples, params=params, active_module=active_module,
                               chunk=P.chunk_points, **render_kwargs)
    return mse_color_loss(pred_rgb, gt_rgb, P.color_space, reduction)


def adapt_step(P, base, rays, rgbs, optimizer, active_module=None, grad_clip: Optional[float] = 1.0,
               group=None, shared: Optional[list] = None, grad_scaler=None, **render_kwargs) -> torch.Tensor:
    """One optimizer update of runtime_adapt (runtime_adapt.py:288-313).  Returns the loss (device).

    ``group`` (expert parallel): ``rays`` / ``rgbs`` are this rank's shard of the global batch, the
    container's experts are distributed over the group (expert_parallel.adapt_step_expert_parallel);
    ``shared`` are the replicated parameters (default: the background head).
    With the use_amp MLP precision (ops.set_train_mlp_precision("amp")) the step runs under a GradScaler as
    the reference's does (runtime_adapt.py:237-268): ``grad_scaler`` (a torch.amp.GradScaler; a fresh one when
    None) scales the loss, unscales, skips a non-finite step and updates its scale."""
    if group is not None and torch.distributed.is_initialized() and torch.distributed.get_world_size(group) > 1:
        from .expert_parallel import HipBackend, adapt_step_expert_parallel
        if active_module is not None:
            raise ValueError("adapt_step: expert-parallel groups adapt the routed container (active_module=None)")
        n = torch.tensor([rays.shape[0]], dtype=torch.int64, device=rays.device)
        torch.distributed.all_reduce(n, group=group)
        shared = list(base.bg_mlp.parameters()) if shared is None else shared
        return adapt_step_expert_parallel(P, HipBackend(base), rays, rgbs, optimizer, len(base.submodules), int(n),
                                          shared, grad_clip=grad_clip, group=group,
                                          u=render_kwargs.get("jitter_u"))
    optimizer.zero_grad()
    loss = compute_mse_loss(P, model=base, data={"rays": rays, "rgbs": rgbs}, params=None,
                            active_module=active_module, reduction="mean", **render_kwargs)
    if ops.TRAIN_MLP_PRECISION == "amp":
        scaler = grad_scaler if grad_scaler is not None else torch.amp.GradScaler("cuda")
        scaler.scale(loss).backward()
        scaler.unscale_(optimizer)
        if isinstance(optimizer, FusedAdam):
            scaler.step(optimizer, max_norm=grad_clip)
        else:
            if grad_clip is not None:
                torch.nn.utils.clip_grad_norm_(base.parameters(), grad_clip)
            scaler.step(optimizer)
        scaler.update()
        return loss.detach()
    loss.backward()
    if isinstance(optimizer, FusedAdam):
        optimizer.step(max_norm=grad_clip)  # clip_grad_norm_ folded into the fused step
    else:
        if grad_clip is not None:
            torch.nn.utils.clip_grad_norm_(base.parameters(), grad_clip)
        optimizer.step()
    return loss.detach()


class GraphedAdaptStep:
    """adapt_step captured once into a HIP graph and replayed per batch (the launch-bound inner loop
    of runtime_adapt: ~165 kernels per 1000-ray step).  Same arithmetic as the eager step -- the Adam
    constants come from FusedAdam's device table, the jitter from the graph-safe generator -- with
    the batch copied into static buffers before each replay.  ``warmup`` eager steps run first (they
    are real updates on the first batch).  Only fixed-shape steps are capturable: one expert
    (``active_module``, the C5 / meta-training placement) or a bare MetaNGP -- the routed container's
    per-expert index selection is data-dependent.  Expert-parallel groups are not captured (use
    adapt_step)."""

    def __init__(self, P, base, rays, rgbs, optimizer, active_module=None, grad_clip: Optional[float] = 1.0,
                 warmup: int = 2, max_steps: int = 1 << 16, **render_kwargs):
        from .meta_container import MetaContainer
        if not isinstance(optimizer, FusedAdam):
            raise TypeError("GraphedAdaptStep needs FusedAdam")
        if isinstance(base, MetaContainer) and active_module is None:
            raise ValueError("GraphedAdaptStep: the routed container step is data-dependent; pass active_module")
        self.static_rays = rays.detach().clone()
        self.static_rgbs = rgbs.detach().clone()
        self.static_u = None
        if render_kwargs.get("jitter_u") is not None:  # caller-supplied jitter: a static input too
            self.static_u = render_kwargs["jitter_u"].detach().clone()
            render_kwargs = dict(render_kwargs, jitter_u=self.static_u)
        self.args = (P, base, optimizer, active_module, grad_clip, render_kwargs)
        side = torch.cuda.Stream(rays.device)
        side.wait_stream(torch.cuda.current_stream(rays.device))
        with torch.cuda.stream(side):
            for _ in range(max(1, int(warmup))):
                adapt_step(P, base, self.static_rays, self.static_rgbs, optimizer, active_module=active_module,
                           grad_clip=grad_clip, **render_kwargs)
        torch.cuda.current_stream(rays.device).wait_stream(side)
        torch.cuda.synchronize(rays.device)
        optimizer.graph_begin(max_steps)
        optimizer.zero_grad(set_to_none=True)
        self.graph = torch.cuda.CUDAGraph()
        with graph_capture(self.graph):
            self.static_loss = adapt_step(P, base, self.static_rays, self.static_rgbs, optimizer,
                                          active_module=active_module, grad_clip=grad_clip, **render_kwargs)
        optimizer.graph_end_capture()
        self.replays = 0
        self.max_steps = int(max_steps)

    def __call__(self, rays: torch.Tensor, rgbs: torch.Tensor, jitter_u: Optional[torch.Tensor] = None) -> torch.Tensor:
        if self.replays >= self.max_steps:
            # past the precomputed Adam table the captured update would silently stop
            raise RuntimeError(f"GraphedAdaptStep: {self.max_steps} replays exhausted the Adam constant table; "
                               f"capture a new GraphedAdaptStep (max_steps=...)")
        self.static_rays.copy_(rays, non_blocking=True)
        self.static_rgbs.copy_(rgbs, non_blocking=True)
        if jitter_u is not None:
            self.static_u.copy_(jitter_u, non_blocking=True)
        self.graph.replay()
        self.replays += 1
        from .optim import bump_versions
        bump_versions(self.args[2]._graph["params"])  # the replayed Adam wrote them: packed images are stale
        return self.static_loss

    def sync_state(self) -> None:
        """Write the replay count into the optimizer's host state['step'] entries."""
        self.args[2].graph_sync_steps(self.replays)


def _routed_step_for(P, model, optimizer, n_rays: int, grad_clip):
    """The RoutedAdaptStep cached on ``optimizer`` for ``model`` (built on first use, sized for the first
    batch), or None when the configuration is outside what the routed pair kernels cover (then the eager
    adapt_step runs).  A batch larger than the cached step's capacity rebuilds it (state carried over
    through the optimizer's host state)."""
    from .meta_container import MetaContainer
    from .routed_train import RoutedAdaptStep
    from ._lib import AcnError
    if not (FAST_RUNTIME_ADAPT and isinstance(model, MetaContainer) and isinstance(optimizer, FusedAdam)):
        return None
    cache = optimizer.__dict__.setdefault("_acn_routed_steps", {})
    key = (id(model), grad_clip, int(P.ray_samples), str(P.color_space))
    st = cache.get(key)
    if st is not None and n_rays <= st.N:
        st.load_state()   # eager steps on this optimizer since the last call advanced the host counters
        return st
    if st is not None:
        st.sync_state()
        del cache[key]
    try:
        st = RoutedAdaptStep(P, model, n_rays, optimizer, grad_clip=grad_clip, graph=True, warmup=1)
    except AcnError:
        return None
    cache[key] = st
    return st


# runtime_adapt's full batches through the cached, graph-replayed RoutedAdaptStep (ACN_FAST_ADAPT=0: the
# eager adapt_step for every batch)
FAST_RUNTIME_ADAPT = os.environ.get("ACN_FAST_ADAPT", "1") != "0"


def runtime_adapt(*, P, model, data_loader: Iterable, optimizer, steps: Optional[int] = None,
                  active_module: Optional[int] = None, grad_clip: Optional[float] = 1.0) -> Dict[str, float]:
    """runtime_adapt.py:213-315: adapt in place; one pass over the loader (steps=None) or exactly
    ``steps`` updates cycling over it.

    The online stage's configuration -- the routed container (``active_module=None``) with FusedAdam --
    runs through one RoutedAdaptStep per (model, optimizer): the first full batch is an eager update, the
    step is then captured and every later batch of that size replays one HIP graph with no host
    synchronisation; a smaller (ragged last) batch runs the same kernels eagerly.  The loss is read once,
    at the end (the reference reads it every step).  Other configurations take the eager adapt_step."""
    device = next(model.parameters()).device
    model.train()
    # the reference clips base.parameters(); parameters outside base get no gradient from the loss
    # (zero_grad sets them to None), so FusedAdam's norm over gradient-carrying tensors is the same
    base = model.submodules[active_module] if active_module is not None else model
    last_loss, step_count = None, 0
    fast = [None, active_module is None]   # [RoutedAdaptStep, still worth trying]
    # use_amp: a fresh GradScaler per call (runtime_adapt.py:237); the cached RoutedAdaptStep's scaler restarts too
    amp = ops.TRAIN_MLP_PRECISION == "amp"
    scaler = torch.amp.GradScaler("cuda") if amp else None
    reset = set()

    def run(rays, rgbs):
        nonlocal last_loss, step_count
        rays, rgbs = rays.to(device, non_blocking=True), rgbs.to(device, non_blocking=True)
        if fast[1] and (fast[0] is None or rays.shape[0] > fast[0].N):
            fast[0] = _routed_step_for(P, base, optimizer, int(rays.shape[0]), grad_clip)
            fast[1] = fast[0] is not None
        if fast[0] is not None:
            if amp and getattr(fast[0], "amp", None) is not None and id(fast[0]) not in reset:
                fast[0].amp.reset()
                reset.add(id(fast[0]))
            last_loss = fast[0](rays, rgbs)
        else:
            last_loss = adapt_step(P, base, rays, rgbs, optimizer, active_module=active_module, grad_clip=grad_clip,
                                   grad_scaler=scaler)
        step_count += 1

    if steps is None:
        for rays, rgbs in data_loader:
            run(rays, rgbs)
    else:
        it = iter(data_loader)
        while step_count < int(steps):
            try:
                rays, rgbs = next(it)
            except StopIteration:
                it = iter(data_loader)
                rays, rgbs = next(it)
            run(rays, rgbs)
    if fast[0] is not None:
        fast[0].sync_state()   # host state['step'] current (state_dict, a later eager step)
    return {"loss": 0.0 if last_loss is None else float(last_loss), "steps": step_count}
