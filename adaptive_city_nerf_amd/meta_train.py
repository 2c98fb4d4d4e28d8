"""Offline meta-training on the HIP path.

Mirrors the reference's pipelines/offline_stage/meta_core.py (``task_adapt`` :14-67, ``meta_update``
:72-123, ``maml_meta_update`` :126-143, ``reptile_meta_update`` :146-182, ``clip_all_grads``
:185-194, ``extract_module_params`` :200-211, ``snapshot_params`` :214-216), the ``train_step`` of
meta_train_step.py:18-253 and the ``compute_loss`` dispatcher of nerfs/losses.py:156-166, with the
same signatures, the same region / task / inner-loop order (so a run consumes training jitter in
the reference's order) and the same loss reductions (sample-weighted region sums, FedAvg scaling by
the number of regions).

Every render goes through the differentiable HIP composition (hash grid forward + scatter-add
backward, MetaLinear chain on rocBLAS, HIP compositing).  Second-order MAML (``create_graph=True``)
runs the inner-loop forwards inside ``ray_rendering.second_order()``, which swaps the compositing to
its twice-differentiable torch form; the hash grid's own backward is never differentiated (fast
weights are the 14 MLP tensors), so it needs no second derivative.  Autocast is not
used: the HIP path computes fp32; a GradScaler passed in is honoured as a scaler.

Differences from the reference, all where the reference cannot run as written:
* Reptile: the reference's train_step calls ``meta_update`` without ``fast_list``
  (meta_train_step.py:168), so Reptile raises TypeError there; and ``reptile_meta_update`` compares
  the expert-relative fast names with the container's meta-parameter names, so it never updates.
  Here train_step collects the adapted fast weights and prefixes them with ``submodules.{cid}.``.
* Expert parallelism (``group``): rank r processes the regions whose expert it owns
  (expert_parallel.expert_owner: contiguous blocks of experts per rank, the same placement as the
  expert-parallel render / adaptation); the region/query counts, the shared background-head
  gradients and the clip norm are all-reduced, so the update equals the single-process one
  (SURVEY §8(e) "Offline meta-training").
"""
from __future__ import annotations

import contextlib
import io
import math
import os
import random
import time
from collections import OrderedDict
from typing import Dict, List, Mapping, Optional

import torch
import torch.distributed as dist

from . import ops
from ._lib import graph_capture
from .expert_parallel import expert_owner, global_clip_grad_norm_
from .encodings import accumulate_table_grad
from .optim import FusedAdam
from .ray_rendering import encoding_frozen, inner_loop_background_cache, second_order
from .train import compute_mse_loss


def psnr(mse):
    return -10.0 * torch.log10(mse + 1e-24)


def to_device_tree(x, device):
    """Recursively move tensors in nested containers to device (common/utils.py:163-175)."""
    if torch.is_tensor(x):
        return x.to(device, non_blocking=True)
    if isinstance(x, Mapping):
        return {k: to_device_tree(v, device) for k, v in x.items()}
    if isinstance(x, (list, tuple)):
        ys = [to_device_tree(v, device) for v in x]
        return tuple(ys) if isinstance(x, tuple) else ys
    return x


def compute_loss(P, model, data, params=None, active_module=None, **kwargs):
    """losses.py:156-166.  With P.fim the reference's compute_fim_loss returns the plain MSE whenever
    the model carries no Fisher store / FIM head (losses.py:78-80) -- the configuration it ships
     -- so both branches are the MSE here."""
    return compute_mse_loss(P, model, data, params, active_module)


# ============================================================================ model helpers
def extract_module_params(submodule, copy=True) -> OrderedDict:
    """Snapshot the submodule's meta-parameters (name -> tensor); copies are fresh leaves (Reptile)."""
    if copy:
        return OrderedDict((n, p.detach().clone().requires_grad_(True)) for n, p in submodule.meta_named_parameters())
    return OrderedDict((n, p) for n, p in submodule.meta_named_parameters())


def snapshot_params(model):
    return {n: p.detach().clone() for n, p in model.meta_named_parameters()}


def snapshot_model_dict(model):
    return {n: p.detach().clone() for n, p in model.state_dict().items()}


# ============================================================================ inner loop
_ONES = {}


def _ones_like_scalar(loss):
    """A persistent 1.0 of the loss's device / dtype as autograd's output gradient (autograd would fill a
    fresh one per backward: one more launch per inner step; the value is the same)."""
    if loss.dim() != 0:
        return None
    key = (loss.device, loss.dtype)
    t = _ONES.get(key)
    if t is None:
        t = _ONES[key] = torch.ones((), device=loss.device, dtype=loss.dtype)
    return t


def task_adapt(P, model, support, inner_lr, iterations, active_module=None):
    """Inner-loop adaptation of the fast weights on a support set (meta_core.py:14-67)."""
    algo = str(getattr(P, "algo", "")).lower()
    first_order = algo in ("fomaml", "reptile")
    base = model.submodules[active_module] if active_module is not None else model
    fast = extract_module_params(base, copy=(algo == "reptile"))
    inner_losses = []
    with inner_loop_background_cache() if first_order else contextlib.nullcontext():
        return _inner_steps(P, model, support, inner_lr, iterations, active_module, first_order, fast, inner_losses)


def _inner_steps(P, model, support, inner_lr, iterations, active_module, first_order, fast, inner_losses):
    """task_adapt's inner gradient steps (meta_core.py:30-64)."""
    for _ in range(int(iterations)):
        with second_order(not first_order), encoding_frozen(first_order):
            loss = compute_loss(P, model, support, params=fast, active_module=active_module, grad_buffer={},
                                update_fisher=True)
        grads = torch.autograd.grad(loss, tuple(fast.values()), grad_outputs=_ones_like_scalar(loss),
                                    create_graph=not first_order, allow_unused=True)
        live = [k for k, g in enumerate(grads) if g is not None]
        if first_order and live:
            # the same w - lr * g (mul, then sub: bitwise equal) as two multi-tensor launches instead of
            # two kernels per tensor; differentiable w.r.t. w for the outer gradient
            names, ws = list(fast.keys()), list(fast.values())
            step = torch._foreach_mul([grads[k].to(ws[k].dtype) for k in live], inner_lr)
            upd = dict(zip(live, torch._foreach_sub([ws[k] for k in live], step)))
            fast = OrderedDict((n, upd.get(k, ws[k])) for k, n in enumerate(names))
        else:
            fast = OrderedDict((n, w if g is None else (w - inner_lr * g.to(w.dtype)))
                               for (n, w), g in zip(fast.items(), grads))
        inner_losses.append(loss.detach())
    return fast, inner_losses


# ============================================================================ outer update
def clip_all_grads(optimizer, grad_clip=1.0, group=None, shared=None):
    """clip_grad_norm_ over every gradient-carrying parameter (meta_core.py:185-194); with an
    expert-parallel ``group`` the norm is global (own experts all-reduced, ``shared`` counted once)."""
    if grad_clip is None:
        return
    params = [p for g in optimizer.param_groups for p in g["params"] if p.grad is not None]
    if not params:
        return
    if group is not None and dist.is_initialized() and dist.get_world_size(group) > 1:
        global_clip_grad_norm_(params, shared or [], grad_clip, group)
    else:
        torch.nn.utils.clip_grad_norm_(params, grad_clip)


def maml_meta_update(optimizer, loss_out, scaler=None, grad_clip=1.0, group=None, shared=None):
    """Outer MAML/FOMAML step (meta_core.py:126-143); FusedAdam folds the clip into its step."""
    if not torch.isfinite(loss_out):
        print(f"[WARN] Skipping meta-update: non-finite loss_out={loss_out.item()}")
        return
    optimizer.zero_grad(set_to_none=True)
    use_amp = scaler is not None and getattr(scaler, "is_enabled", lambda: False)()
    if use_amp:
        scaler.scale(loss_out).backward()
        scaler.unscale_(optimizer)
        _allreduce_shared_grads(shared, group)
        clip_all_grads(optimizer, grad_clip, group, shared)
        scaler.step(optimizer)
        scaler.update()
        return
    loss_out.backward()
    _allreduce_shared_grads(shared, group)
    if isinstance(optimizer, FusedAdam):
        if shared:
            optimizer.shared_params = {id(p) for p in shared}
        optimizer.step(max_norm=grad_clip, sumsq_group=group)
    else:
        clip_all_grads(optimizer, grad_clip, group, shared)
        optimizer.step()


@torch.no_grad()
def reptile_meta_update(P, model, fast_list):
    """theta <- theta + lr * mean_i(W_i - theta) over the meta-parameters (meta_core.py:146-182)."""
    if fast_list is None or len(fast_list) == 0:
        raise ValueError("Reptile update called with empty fast_list")
    theta = snapshot_params(model)
    sum_delta = {k: torch.zeros_like(v) for k, v in theta.items()}
    for fast in fast_list:
        for k, v in fast.items():
            if k in sum_delta:
                sum_delta[k].add_(v.detach() - theta[k])
    n = float(len(fast_list))
    updated = []
    for name, p in model.meta_named_parameters():
        if name in sum_delta:
            delta = sum_delta[name] / n
            if torch.isfinite(delta).all() and delta.abs().sum() > 0:
                p.add_(P.lr * delta)
                updated.append(name)
    print("Reptile meta-update: updated %d parameter tensors: %s" % (len(updated), ", ".join(updated) or "<none>"))


def meta_update(P, model, optimizer, loss_out, scheduler=None, grad_scaler=None, fast_list=None, group=None,
                shared=None, verbose=True):
    """Unified outer update (meta_core.py:72-123)."""
    algo = P.algo.lower()
    if algo in ("maml", "fomaml"):
        maml_meta_update(optimizer, loss_out, scaler=grad_scaler, grad_clip=getattr(P, "grad_clip", 1.0),
                         group=group, shared=shared)
    elif algo == "reptile":
        reptile_meta_update(P, model, fast_list=fast_list)
    else:
        raise ValueError(f"Unsupported algo {algo!r}")
    if verbose:
        with torch.no_grad():  # per-region outer gradient norms, one device->host copy
            norms = []
            for expert in model.submodules:
                sq = [p.grad.double().pow(2).sum() for p in expert.parameters() if p.grad is not None]
                norms.append(torch.stack(sq).sum() if sq else torch.zeros((), dtype=torch.float64,
                                                                           device=loss_out.device))
            for cid, v in enumerate(torch.stack(norms).sqrt().tolist()):
                print(f"debug/outer_grad_norm_region_{cid}: ", v)
    if scheduler is not None:
        scheduler.step()
    if verbose:
        print(f"group LRs = {[g['lr'] for g in optimizer.param_groups]}")


def _allreduce_shared_grads(shared, group):
    """Sum the shared (background-head) gradients over the expert-parallel group."""
    if group is None or not dist.is_initialized() or dist.get_world_size(group) <= 1 or not shared:
        return
    grads = [p.grad for p in shared if p.grad is not None]
    if not grads:
        return
    flat = torch.cat([g.reshape(-1) for g in grads])
    dist.all_reduce(flat, group=group)
    off = 0
    for g in grads:
        g.copy_(flat[off: off + g.numel()].view_as(g))
        off += g.numel()


@torch.no_grad()
def broadcast_experts(model, group=None):
    """Expert parallelism: copy every expert's parameters and buffers from its owner rank
    (expert_owner) to all ranks (e.g. before evaluation or a checkpoint)."""
    if not dist.is_initialized() or dist.get_world_size(group) <= 1:
        return
    world = dist.get_world_size(group)
    owner = expert_owner(len(model.submodules), world)
    for cid, expert in enumerate(model.submodules):
        src = dist.get_global_rank(group, owner[cid]) if group is not None else owner[cid]
        for t in list(expert.parameters()) + list(expert.buffers()):
            dist.broadcast(t.data, src=src, group=group)


# ============================================================================ one meta step
# train_step's FOMAML steps through the cached GraphedMetaStep (ACN_FAST_META=0: the eager step every time)
FAST_META_STEP = os.environ.get("ACN_FAST_META", "1") != "0"
# Visit each task's support and query rays in ray_order_kernel's direction-cell order (one permutation of the
# task's rays and colours per outer step, before its inner loop).  The reference draws a task's rays at random
# (task_dataset.py), so the order of rays inside a task carries no meaning; the losses are means over rays
# (equal up to fp summation order).  The hash-grid gathers of the 8 inner renders and the query render then
# see neighbouring rays together.
TASK_RAY_ORDER = os.environ.get("ACN_META_TASK_ORDER", "0") != "0"


def _ordered_part(part: Mapping[str, torch.Tensor]) -> Dict[str, torch.Tensor]:
    """{"rays", "rgbs"} of one task part in direction-cell order (TASK_RAY_ORDER), or unchanged."""
    rays = part["rays"]
    n = int(rays.shape[0])
    if not TASK_RAY_ORDER or not rays.is_cuda or n < 2 or n > 8192:
        return part
    from .ray_rendering import _train_order
    order, _ = _train_order(rays)
    out = dict(part)
    out["rays"] = rays.index_select(0, order)
    out["rgbs"] = part["rgbs"].index_select(0, order)
    return out


def _graph_eligible(P, model, optimizer, scheduler, grad_scaler, group) -> bool:
    if not FAST_META_STEP or str(getattr(P, "algo", "")).lower() != "fomaml" or not isinstance(optimizer, FusedAdam):
        return False
    if grad_scaler is not None and getattr(grad_scaler, "is_enabled", lambda: False)() and \
            ops.TRAIN_MLP_PRECISION != "amp":
        return False   # a GradScaler is replayed on the device with the use_amp kernels (GraphedMetaStep.amp)
    if group is not None and dist.is_initialized() and dist.get_world_size(group) > 1:
        return False
    return hasattr(model, "submodules") and not getattr(model, "use_occ", False)


def train_step(P, step, model, optimizer, task_data, metric_logger=None, logger=None, scheduler=None,
               grad_scaler=None, group=None):
    """One offline meta-training step over tasks grouped by region (meta_train_step.py:18-253).

    ``task_data``: {cid: [task, ...]} with task.support / task.query (or dict keys) holding
    {"rays": (n, 8), "rgbs": (n, 3)}.  Returns a dict of the step's losses and timings.

    FOMAML on one process with FusedAdam (the reference's configs/train.json setup) goes through a
    GraphedMetaStep cached on the optimizer: the first call is the eager step, after which the per-region
    task graphs and the outer update are captured, and later calls replay them (a step whose task shapes
    the graphs do not cover runs eagerly inside it).  The replayed step skips meta_update's per-region
    debug prints.  Everything else (MAML, Reptile, expert-parallel groups, a GradScaler) is eager."""
    out = None
    g = optimizer.__dict__.get("_acn_meta_graph") if _graph_eligible(P, model, optimizer, scheduler, grad_scaler,
                                                                      group) else False
    if g == "pending":   # second eligible call: capture now (the first call's gradients stayed readable)
        try:
            g = optimizer._acn_meta_graph = GraphedMetaStep(P, model, optimizer, task_data, warmup=0,
                                                            grad_scaler=grad_scaler)
        except (ValueError, TypeError):
            g = optimizer._acn_meta_graph = False   # shapes the graphs cannot cover: stay eager
    if isinstance(g, GraphedMetaStep):
        out = g(step, task_data)
        # host state['step'] (and the first-updated experts' state entries) current after every replayed step:
        # optimizer.state_dict() -- the reference's checkpoint (utils.py:290) -- sees the real counts
        g.sync_state()
        if out is not None and scheduler is not None:
            scheduler.step()
    else:
        g_prev = optimizer.__dict__.get("_acn_meta_graph")
        if isinstance(g_prev, GraphedMetaStep):
            # an ineligible call (a GradScaler, MAML ...) on an optimizer a graphed step also updates: hand the
            # state over both ways, as GraphedMetaStep._eager does
            g_prev.adam.sync_state(extra_slots=set(range(g_prev.adam.nslots)))
        out = _train_step_eager(P, step, model, optimizer, task_data, scheduler, grad_scaler, group, logger)
        if isinstance(g_prev, GraphedMetaStep):
            g_prev.adam.load_state()
        if g is None:
            optimizer._acn_meta_graph = "pending"
    if out is None:
        return None
    for k in ("time_setup", "time_data", "time_inner", "time_outer", "time_misc"):
        out.setdefault(k, 0.0)
    if metric_logger is not None:
        metric_logger.meters["batch_time"].update(out["time_total_step"], n=1)
        metric_logger.meters["tasks"].update(out["tasks"], n=1)
        metric_logger.meters["loss_in"].update(out["loss_in"], n=out["rays_in"])
        metric_logger.meters["psnr_in"].update(out["psnr_in"], n=out["rays_in"])
        metric_logger.meters["loss_out"].update(out["loss_out"], n=out["rays_out"])
        metric_logger.meters["psnr_out"].update(out["psnr_out"], n=out["rays_out"])
        if hasattr(metric_logger, "synchronize_between_processes"):
            metric_logger.synchronize_between_processes()
    if logger is not None and step % getattr(P, "print_step", 1) == 0:
        logger.log_dirname(f"Step {step}")
        for k in ("loss_in", "loss_out", "psnr_in", "psnr_out"):
            logger.scalar_summary(f"train/{k}", out[k], step)
        for k in ("time_setup", "time_data", "time_inner", "time_outer", "time_misc", "time_total_step"):
            logger.scalar_summary(f"train/{k}", out[k], step)
        logger.log("[TRAIN] [Step %d] [LossIn %.6f] [LossOut %.6f] [PSNRIn %.2f] [PSNROut %.2f] [InnerLR %.6f]"
                   % (step, out["loss_in"], out["loss_out"], out["psnr_in"], out["psnr_out"], float(P.inner_lr)))
    return out


def _train_step_eager(P, step, model, optimizer, task_data, scheduler=None, grad_scaler=None, group=None,
                      logger=None):
    """The eager body of train_step (meta_train_step.py:18-253) without the metric / logger updates."""
    t_step_start = time.perf_counter()
    model.train()
    device = next(model.parameters()).device
    time_setup = time_data = time_inner = time_outer = 0.0
    t0 = time.perf_counter()
    total_tasks = sum(len(v) for v in task_data.values())
    cids = list(task_data.keys())
    rnd = random.Random(getattr(P, "seed", 0) + step)
    rnd.shuffle(cids)
    num_regions = len(cids)
    world, rank = 1, 0
    if group is not None and dist.is_initialized():
        world, rank = dist.get_world_size(group), dist.get_rank(group)
    owner = expert_owner(len(model.submodules), world) if hasattr(model, "submodules") else [0] * (max(cids) + 1)
    mine = [cid for cid in cids if owner[cid] == rank]
    region_inner_sum = {cid: torch.tensor(0.0, device=device) for cid in cids}
    region_inner_count = {cid: 0 for cid in cids}
    region_query_sum = {cid: torch.tensor(0.0, device=device) for cid in cids}
    region_query_count = {cid: 0 for cid in cids}
    algo = str(getattr(P, "algo", "")).lower()
    fast_list: List[Dict[str, torch.Tensor]] = []
    time_setup += time.perf_counter() - t0

    for cid in mine:
        for task in task_data[cid]:
            t1 = time.perf_counter()
            if hasattr(task, "support") and hasattr(task, "query"):
                sup_i, qry_i = task.support, task.query
            else:
                sup_i, qry_i = task["support"], task["query"]
            sup_i = _ordered_part(to_device_tree(sup_i, device))
            qry_i = _ordered_part(to_device_tree(qry_i, device))
            time_data += time.perf_counter() - t1
            n_sup, n_q = int(sup_i["rays"].shape[0]), int(qry_i["rays"].shape[0])
            if n_sup == 0 or n_q == 0:
                if logger is not None:
                    logger.log(f"[WARN] Empty task in region {cid}; skipping.")
                continue
            t2 = time.perf_counter()
            fast_i, inner_losses = task_adapt(P, model, sup_i, P.inner_lr, P.inner_iter, active_module=cid)
            time_inner += time.perf_counter() - t2
            last_inner = inner_losses[-1] if inner_losses else torch.tensor(0.0, device=device)
            region_inner_sum[cid] += last_inner.detach() * n_sup
            region_inner_count[cid] += n_sup
            if algo == "reptile":
                fast_list.append({f"submodules.{cid}.{n}": v for n, v in fast_i.items()})
            t3 = time.perf_counter()
            loss_q = compute_loss(P, model, qry_i, params=fast_i, active_module=cid)
            time_outer += time.perf_counter() - t3
            region_query_sum[cid] += loss_q * n_q
            region_query_count[cid] += n_q

    total_sup = sum(region_inner_count.values())
    total_q = sum(region_query_count.values())
    if world > 1:  # global sample counts
        c = torch.tensor([float(total_sup), float(total_q)], device=device, dtype=torch.float64)
        dist.all_reduce(c, group=group)
        total_sup, total_q = int(c[0]), int(c[1])
    if total_q == 0:
        if logger is not None:
            logger.log("[WARN] train_step_ray: no query samples in any region; skipping step")
        return None
    loss_in_local = sum(region_inner_sum[cid] for cid in cids) / max(total_sup, 1)
    loss_out_local = sum(region_query_sum[cid] for cid in cids) / total_q
    loss_out_meta = num_regions * loss_out_local  # FedAvg scaled by regions (meta_train_step.py:157-159)

    t4 = time.perf_counter()
    shared = list(model.bg_mlp.parameters()) if getattr(model, "use_bg_nerf", False) else None
    meta_update(P, model, optimizer, loss_out_meta, scheduler=scheduler, grad_scaler=grad_scaler,
                fast_list=fast_list if algo == "reptile" else None, group=group if world > 1 else None,
                shared=shared)
    time_outer += time.perf_counter() - t4
    if getattr(model, "use_occ", False):
        model.maybe_update_expert_occupancies(step, params=None)
    if torch.cuda.is_available():
        torch.cuda.synchronize()

    loss_in, loss_out = loss_in_local.detach(), loss_out_local.detach()
    if world > 1:
        s = torch.stack([loss_in.double(), loss_out.double()])
        dist.all_reduce(s, group=group)
        loss_in, loss_out = s[0].float(), s[1].float()
    t_total = time.perf_counter() - t_step_start
    t_misc = max(0.0, t_total - (time_setup + time_data + time_inner + time_outer))
    return {"loss_in": float(loss_in), "loss_out": float(loss_out), "psnr_in": float(psnr(loss_in)),
            "psnr_out": float(psnr(loss_out)), "tasks": total_tasks, "rays_in": total_sup, "rays_out": total_q,
            "time_setup": time_setup, "time_data": time_data, "time_inner": time_inner, "time_outer": time_outer,
            "time_misc": t_misc, "time_total_step": t_total}


# ============================================================================ graph-replayed meta step
class GraphedMetaStep:
    """train_step for FOMAML with every region's task processing replayed as a HIP graph.

    The outer loss of meta_train_step.py:157-159 is ``R * sum_t n_q,t loss_q,t / total_q`` over the
    step's tasks, so its gradient is the sum of per-task gradients weighted by ``R n_q,t / total_q``:
    each task's inner loop (task_adapt, meta_core.py:14-67), query loss and backward (into persistent
    gradient buffers) is one captured graph per region (the expert and the task shapes are fixed per
    region), replayed for every task of the region in the reference's shuffled region order
    (random.Random(seed + step)); the training jitter is drawn inside the graphs (graph-safe philox) in the
    same call order.  The outer clip + Adam is one more graph on optim.SlottedAdam: expert k is updated
    only when region k processed a task this step (a per-step activity vector the host writes), with its
    own device step counter -- torch.optim.Adam skips a parameter whose .grad is None, and an expert whose
    region has no tasks gets none (meta_core.py:126-143).  Per step the host copies each task into its
    region's static buffers and reads the loss once (the reference's non-finite-loss skip,
    meta_core.py:124-126).  Empty tasks are skipped as the reference skips them; a task whose non-empty
    shapes differ from the captured ones, or a region that was not captured, sends that step through the
    eager train_step (state carried over in both directions).  The gradient equals the eager step's up to
    fp32 summation order (per-task accumulation instead of one backward of the sum).  Second-order MAML
    stays on the eager train_step: the create_graph backward does an operation HIP stream capture does not
    permit on this stack."""

    def __init__(self, P, model, optimizer, task_data, warmup: int = 1, max_steps: int = 1 << 16,
                 grad_scaler=None):
        algo = str(getattr(P, "algo", "")).lower()
        if algo != "fomaml":
            raise ValueError("GraphedMetaStep: FOMAML only (MAML's second-order backward is not capturable; "
                             "Reptile has no gradient step) -- use train_step")
        if not isinstance(optimizer, FusedAdam):
            raise TypeError("GraphedMetaStep needs FusedAdam (its slotted device step makes the update replayable)")
        from .optim import AmpScaler, SlottedAdam
        self.P, self.model, self.opt = P, model, optimizer
        self.device = next(model.parameters()).device
        # use_amp (meta_core.py:123-136 with trainer.py:24's GradScaler): the query loss is scaled by the
        # scaler's device scale inside the task graphs and the outer graph unscales / skips / updates it, on
        # the GradScaler's own state tensors (its get_scale() and state_dict() follow the replays)
        self.amp = AmpScaler.wrap(grad_scaler, self.device) if grad_scaler is not None and \
            getattr(grad_scaler, "is_enabled", lambda: False)() else None
        self.grad_scaler = grad_scaler if self.amp is not None else None
        self.shapes = {}
        for cid, tasks in task_data.items():
            for t in tasks:
                ns, nq = _task_shapes(t)
                if ns == 0 or nq == 0:
                    continue
                if self.shapes.setdefault(cid, (ns, nq)) != (ns, nq):
                    raise ValueError(f"GraphedMetaStep: region {cid} has tasks of different shapes")
        self.cids = sorted(self.shapes)
        if not self.cids:
            raise ValueError("GraphedMetaStep: no non-empty task to capture")
        for _ in range(max(0, int(warmup))):   # real updates
            with _quiet():
                _train_step_eager(P, 0, model, optimizer, task_data, grad_scaler=self.grad_scaler)
        torch.cuda.synchronize(self.device)
        dev = self.device
        self.static = {}
        self.inner_acc = torch.zeros((), device=dev)
        self.q_acc = torch.zeros((), device=dev)
        K = len(model.submodules)
        slot_of = {}
        for k, sub in enumerate(model.submodules):
            for p in sub.parameters():
                slot_of[id(p)] = k
        for p in model.parameters():
            slot_of.setdefault(id(p), K)          # the shared background head
        self.params = [p for g in optimizer.param_groups for p in g["params"] if id(p) in slot_of]
        for p in self.params:   # persistent gradients: the captured backwards accumulate into them
            p.grad = torch.zeros_like(p)
        self.grads = [p.grad for p in self.params]
        self.adam = SlottedAdam(optimizer, slot_of, {id(p): p.grad for p in self.params}, K, K + 1,
                                max_steps=max_steps)
        self.K = K
        # activity of the outer update: seg[K + 1 + k] > 0 <=> region k processed a task (SlottedAdam)
        self.act = torch.zeros(2 * K + 1, dtype=torch.int64, device=dev)
        self.act_host = torch.zeros(2 * K + 1, dtype=torch.int64).pin_memory()
        self.pool = torch.cuda.graph_pool_handle()
        self.graphs = {}
        for cid in self.cids:
            self._add_region(cid, next(t for t in task_data[cid] if _task_shapes(t) == self.shapes[cid]))
        self.outer = torch.cuda.CUDAGraph()
        with graph_capture(self.outer, pool=self.pool):
            self.adam.step(self.act, getattr(P, "grad_clip", 1.0), amp=self.amp)
        self.replays = 0
        self.eager_steps = 0
        torch._foreach_zero_(self.grads)

    def _add_region(self, cid, task) -> None:
        """Static buffers + the captured task graph of region ``cid`` at the shapes of ``task`` (capture runs
        nothing; a region first seen after construction is added the same way)."""
        dev = self.device
        ns, nq = _task_shapes(task)
        self.shapes[cid] = (ns, nq)
        self.static[cid] = {"support": {"rays": torch.zeros(ns, 8, device=dev), "rgbs": torch.zeros(ns, 3, device=dev)},
                            "query": {"rays": torch.zeros(nq, 8, device=dev), "rgbs": torch.zeros(nq, 3, device=dev)},
                            "wq": torch.zeros((), device=dev)}
        self._load(cid, task)
        sub = self.model.submodules[cid] if hasattr(self.model, "submodules") else None
        if sub is not None and hasattr(sub, "_host_box"):
            sub._host_box()   # host-side box cache filled outside the capture (a region first seen now)
        torch.cuda.synchronize(dev)
        g = torch.cuda.CUDAGraph()
        with graph_capture(g, pool=self.pool):
            self._task(cid)
        self.graphs[cid] = g

    def _load(self, cid, task) -> None:
        sup, qry = (task.support, task.query) if hasattr(task, "support") else (task["support"], task["query"])
        st = self.static[cid]
        for part, src in (("support", sup), ("query", qry)):
            if src["rays"].shape[0] == st[part]["rays"].shape[0]:
                src = _ordered_part(src)
            if src["rays"].shape[0] != st[part]["rays"].shape[0]:
                raise ValueError(f"GraphedMetaStep: region {cid} was captured for {st[part]['rays'].shape[0]} "
                                 f"{part} rays, got {src['rays'].shape[0]}")
            st[part]["rays"].copy_(src["rays"], non_blocking=True)
            st[part]["rgbs"].copy_(src["rgbs"], non_blocking=True)

    def _task(self, cid) -> None:
        P, st = self.P, self.static[cid]
        ns, nq = self.shapes[cid]
        fast, inner = task_adapt(P, self.model, st["support"], P.inner_lr, P.inner_iter, active_module=cid)
        loss_q = compute_loss(P, self.model, st["query"], params=fast, active_module=cid)
        # the task's outer gradient added into the persistent .grad buffers: the table scatter adds into
        # its buffer directly (encodings.accumulate_table_grad), the other tensors with one multi-tensor
        # add instead of an AccumulateGrad launch each (same sums as .backward())
        targets = self.params   # every optimised tensor (those the task does not reach come back None)
        with accumulate_table_grad():
            lq = loss_q * st["wq"] if self.amp is None else loss_q * st["wq"] * self.amp.scale   # scaler.scale
            gs = torch.autograd.grad(lq, targets, grad_outputs=_ones_like_scalar(lq), allow_unused=True)
        live = [(p.grad, g) for p, g in zip(targets, gs) if g is not None]
        if live:
            torch._foreach_add_([a for a, _ in live], [b for _, b in live])
        if inner:
            self.inner_acc.add_(inner[-1].detach() * ns)
        self.q_acc.add_(loss_q.detach() * nq)

    def _covers(self, task_data) -> bool:
        """Every non-empty task has its region's captured shapes; a region seen for the first time (with one
        task shape, of an expert of the container) gets its graph captured here."""
        new_shape, new_task = {}, {}
        for cid, tasks in task_data.items():
            for t in tasks:
                sh = _task_shapes(t)
                if sh[0] == 0 or sh[1] == 0:
                    continue   # skipped, as the reference skips empty tasks
                want = self.shapes.get(cid, new_shape.get(cid))
                if want is None and isinstance(cid, int) and 0 <= cid < self.K:
                    new_shape[cid], new_task[cid] = sh, t
                    want = sh
                if want != sh:
                    return False
        for cid, t in new_task.items():
            self._add_region(cid, t)
        return True

    def _eager(self, step, task_data):
        """A step the graphs do not cover: the eager train_step on the same optimizer, state carried over."""
        live = [c for c, ts in task_data.items() if any(min(_task_shapes(t)) > 0 for t in ts)]
        self.adam.sync_state(extra_slots=set(live) | {self.K})   # the slots the eager step will update
        for p in self.params:
            p.grad = None
        with _quiet():
            out = _train_step_eager(self.P, step, self.model, self.opt, task_data, grad_scaler=self.grad_scaler)
        self.adam.load_state()
        for p, g in zip(self.params, self.grads):
            p.grad = g
        torch._foreach_zero_(self.grads)
        self.eager_steps += 1
        return out

    def __call__(self, step: int, task_data) -> Optional[Dict[str, float]]:
        if not self._covers(task_data):
            return self._eager(step, task_data)
        t0 = time.perf_counter()
        torch._foreach_zero_(self.grads)
        self.inner_acc.zero_()
        self.q_acc.zero_()
        cids = list(task_data.keys())
        random.Random(getattr(self.P, "seed", 0) + step).shuffle(cids)
        live = {c: [t for t in task_data[c] if min(_task_shapes(t)) > 0] for c in cids}
        total_sup = sum(self.shapes[c][0] * len(live[c]) for c in cids if live[c])
        total_q = sum(self.shapes[c][1] * len(live[c]) for c in cids if live[c])
        if total_q == 0:
            return None
        self.adam.refresh()   # an LR scheduler may have changed the groups since the last step
        for cid in cids:
            if not live[cid]:
                continue
            self.static[cid]["wq"].fill_(len(cids) * self.shapes[cid][1] / total_q)
            for task in live[cid]:
                self._load(cid, task)
                self.graphs[cid].replay()
        loss_out = float(self.q_acc) / total_q          # the one host read of the step
        if not math.isfinite(len(cids) * loss_out):
            print(f"[WARN] Skipping meta-update: non-finite loss_out={len(cids) * loss_out}")
        else:
            self.act_host.zero_()
            for cid in cids:
                if live[cid]:
                    self.act_host[self.K + 1 + cid] = 1
            self.act.copy_(self.act_host, non_blocking=True)
            self.outer.replay()
            self.replays += 1
            from .optim import bump_versions
            bump_versions([r[0] for r in self.adam.rows])
        loss_in = float(self.inner_acc) / max(total_sup, 1)
        return {"loss_in": loss_in, "loss_out": loss_out, "psnr_in": -10.0 * math.log10(loss_in + 1e-24),
                "psnr_out": -10.0 * math.log10(loss_out + 1e-24), "tasks": sum(len(v) for v in task_data.values()),
                "rays_in": total_sup, "rays_out": total_q, "time_total_step": time.perf_counter() - t0}

    @property
    def last_norm(self) -> torch.Tensor:
        return self.adam.scale

    def sync_state(self) -> None:
        """Host state['step'] of every parameter from the per-slot device counters (state_dict)."""
        self.adam.sync_state()


def _task_shapes(task):
    sup, qry = (task.support, task.query) if hasattr(task, "support") else (task["support"], task["query"])
    return int(sup["rays"].shape[0]), int(qry["rays"].shape[0])


@contextlib.contextmanager
def _quiet():
    with contextlib.redirect_stdout(io.StringIO()):
        yield
