"""Optimizer step of the online adaptation loop on the HIP kernels of csrc/optim.hip.

Reference: ``torch.nn.utils.clip_grad_norm_(base.parameters(), grad_clip)`` then
``optimizer.step()`` with ``torch.optim.Adam(param_groups)`` (pipelines/online_stage/
runtime_adapt.py:305-309, common/utils.py:16-62).  ``FusedAdam`` keeps torch.optim.Adam's
constructor, param-group and state layout (``state[p] = {"step", "exp_avg", "exp_avg_sq"}``, so
state dicts load either way) but performs the whole step -- every tensor of every group -- in one
multi-tensor launch, optionally with the clip coefficient of ``clip_grad_norm_`` folded in
(``step(max_norm=...)``: norm -> coefficient -> update, three launches, no host synchronisation).
There is no CPU path: parameters must live on a HIP device.
"""
from __future__ import annotations

import ctypes as C
import os
from typing import Iterable, Optional

import torch
import torch.distributed as dist

from . import _lib
from ._lib import ACN_OPTIM_CHUNK, ACN_OPTIM_MAX_GROUPS, AcnError, acn_adam_group, check, require_hip


class _Plan:
    """Device descriptors (acn_param_desc) + chunk -> tensor map for a list of (p, g, m, v, key).
    Under stream capture the descriptors travel as kernel arguments (acn_optim_plan_device)."""

    def __init__(self, rows, device):
        if torch.cuda.is_current_stream_capturing() and rows:
            self._init_captured(rows, device)
            return
        self.key = tuple((p.data_ptr(), 0 if g is None else g.data_ptr(), m.data_ptr(), v.data_ptr(), k)
                         for p, g, m, v, k in rows)
        descs, owners, first = [], [], 0
        for t, (p, g, m, v, k) in enumerate(rows):
            n = p.numel()
            nch = (n + ACN_OPTIM_CHUNK - 1) // ACN_OPTIM_CHUNK
            descs.append([p.data_ptr(), 0 if g is None else g.data_ptr(), m.data_ptr(), v.data_ptr(), n,
                          (first << 32) | k])
            owners.append(torch.full((nch,), t, dtype=torch.int32))
            first += nch
        self.nchunks = first
        host = torch.tensor(descs, dtype=torch.int64).pin_memory() if descs else torch.zeros(0, 6, dtype=torch.int64)
        self.descs = host.to(device, non_blocking=True)
        own = torch.cat(owners) if owners else torch.zeros(0, dtype=torch.int32)
        self.chunk_tensor = own.pin_memory().to(device, non_blocking=True) if own.numel() else own.to(device)
        self.partials = torch.empty(max(first, 1), dtype=torch.float64, device=device)
        self._keep = (host, own)

    def _init_captured(self, rows, device):
        self.key = tuple((p.data_ptr(), 0 if g is None else g.data_ptr(), m.data_ptr(), v.data_ptr(), k)
                         for p, g, m, v, k in rows)
        arr = (_lib.acn_param_desc * len(rows))()
        first = 0
        for t, (p, g, m, v, k) in enumerate(rows):
            arr[t] = _lib.acn_param_desc(p.data_ptr(), 0 if g is None else g.data_ptr(), m.data_ptr(), v.data_ptr(),
                                         p.numel(), k, first)
            first += (p.numel() + ACN_OPTIM_CHUNK - 1) // ACN_OPTIM_CHUNK
        self.nchunks = first
        self.descs = torch.empty(len(rows) * C.sizeof(_lib.acn_param_desc), dtype=torch.uint8, device=device)
        self.chunk_tensor = torch.empty(max(first, 1), dtype=torch.int32, device=device)
        self.partials = torch.empty(max(first, 1), dtype=torch.float64, device=device)
        check(_lib.lib().acn_optim_plan_device(arr, len(rows), self.descs.data_ptr(), self.chunk_tensor.data_ptr(),
                                               first, _stream(device)), "acn_optim_plan_device")
        self._keep = (arr,)


# Optional timing hook (bench.py): when set to a list, FusedAdam.step appends a pair of recorded
# HIP events bracketing exactly the Adam launch on the current stream.
EVENT_HOOK = None
# SlottedAdam: the clip norm's partial sums, their reduction and the clip coefficient in one launch
# (acn_grad_clip_slots) instead of three; bitwise the same (tests/test_routed_glue.py)
FUSED_CLIP = os.environ.get("ACN_FUSED_CLIP", "1") != "0"


def bump_versions(params) -> None:
    """The kernels write parameters through raw pointers, which torch does not see: bump the
    version counters so caches keyed on them (ops.PackCache, the packed MLP image of the fused
    render) notice the update, as torch.optim.Adam's in-place ops would."""
    if params:
        torch.autograd.graph.increment_version(list(params))


def _stream(device) -> int:
    return int(torch.cuda.current_stream(device).cuda_stream)


def grad_sumsq(params, device, plan: Optional[_Plan] = None) -> torch.Tensor:
    """Sum of squared gradients of ``params`` as a 1-element float64 device tensor."""
    if plan is None:
        rows = [(p, p.grad, p, p, 0) for p in params if p.grad is not None]
        plan = _Plan(rows, device)
    total = torch.empty(1, dtype=torch.float64, device=device)
    check(_lib.lib().acn_grad_sumsq(plan.descs.data_ptr() if plan.nchunks else None,
                                    plan.chunk_tensor.data_ptr() if plan.nchunks else None, plan.nchunks,
                                    plan.partials.data_ptr(), total.data_ptr(), _stream(device)), "acn_grad_sumsq")
    return total


def clip_coef(total_sumsq: torch.Tensor, max_norm: float) -> torch.Tensor:
    """(total_norm, clip coefficient) as a 2-element float32 device tensor."""
    out = torch.empty(2, dtype=torch.float32, device=total_sumsq.device)
    check(_lib.lib().acn_clip_coef(total_sumsq.data_ptr(), float(max_norm), out.data_ptr(),
                                   _stream(total_sumsq.device)), "acn_clip_coef")
    return out


def clip_grad_norm_(parameters, max_norm: float, norm_type: float = 2.0, group=None) -> torch.Tensor:
    """torch.nn.utils.clip_grad_norm_ (2-norm) with the norm reduced by one HIP launch pair;
    gradients are scaled in place.  ``group``: all-reduce the squared norm over ranks first."""
    if norm_type != 2.0:
        raise AcnError("clip_grad_norm_: only the 2-norm (the reference's) is implemented on the HIP path")
    params = [p for p in (parameters if not isinstance(parameters, torch.Tensor) else [parameters])]
    grads = [p.grad for p in params if p.grad is not None]
    if not grads:
        return torch.tensor(0.0)
    device = grads[0].device
    require_hip(grads[0], "clip_grad_norm_")
    total = grad_sumsq([p for p in params if p.grad is not None], device)
    if group is not None and dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.all_reduce(total, group=group)
    nc = clip_coef(total, max_norm)
    torch._foreach_mul_(grads, nc[1])
    return nc[0]


class FusedAdam(torch.optim.Optimizer):
    """torch.optim.Adam (amsgrad=False, maximize=False) as one multi-tensor HIP step."""

    def __init__(self, params, lr: float = 1e-3, betas=(0.9, 0.999), eps: float = 1e-8, weight_decay: float = 0.0,
                 amsgrad: bool = False, **unused):
        if amsgrad:
            raise AcnError("FusedAdam: amsgrad is not implemented (the reference does not use it)")
        defaults = dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay, amsgrad=False, maximize=False,
                        foreach=None, capturable=False, differentiable=False, fused=None)
        super().__init__(params, defaults)
        self._plan = None
        self._splans = None
        self.last_norm: Optional[torch.Tensor] = None   # (total_norm, coef) of the last clipped step
        # parameters replicated across an expert-parallel group (e.g. the shared background head):
        # their squared norm is added once, after the all-reduce of everyone else's
        self.shared_params = set()
        self._graph = None   # graph-replay state (GraphedAdaptStep): device step counter + constant table

    # ------------------------------------------------------------------ graph replay
    def graph_begin(self, max_steps: int = 1 << 16) -> None:
        """Prepare a capture: the Adam constants of the next ``max_steps`` steps go to a device table and
        the step count to a device counter, so the captured update is right on every replay
        (acn_adam_step_table).  The captured step must find every gradient-carrying parameter at the
        step after the highest one recorded now (run the warmup steps first)."""
        cur = 0
        for group in self.param_groups:
            for p in group["params"]:
                st = self.state.get(p)
                if st and "step" in st:
                    cur = max(cur, int(st["step"].item()))
        ng = len(self.param_groups)
        L = _lib.lib()
        nbytes = int(L.acn_adam_table_bytes(ng, int(max_steps)))
        host = torch.empty(nbytes, dtype=torch.uint8)
        groups = (acn_adam_group * ng)()
        for i, g in enumerate(self.param_groups):
            b1, b2 = g["betas"]
            groups[i] = acn_adam_group(float(g["lr"]), float(b1), float(b2), float(g["eps"]), float(g["weight_decay"]),
                                       cur + 1, 0)
        check(L.acn_adam_table_fill(groups, ng, cur + 1, int(max_steps), host.data_ptr(), nbytes),
              "acn_adam_table_fill")
        device = next(p for g in self.param_groups for p in g["params"]).device
        self._graph = {"table": host.to(device), "step_dev": torch.tensor([cur], dtype=torch.int32, device=device),
                       "first": cur + 1, "steps": int(max_steps), "params": []}
        rows, _ = self._rows(bump=False)   # the descriptors, built now with plain copies (no 64-tensor
        if rows:                           # kernel-argument limit inside the capture)
            self._plan = _Plan(rows, device)

    def graph_end_capture(self) -> None:
        """After the capture: undo the host-side step increments the capture pass made."""
        self.graph_sync_steps(0)

    def graph_sync_steps(self, replays: int) -> None:
        """Host-side state['step'] of the captured parameters after ``replays`` replays (state_dict)."""
        gs = self._graph
        for p in gs["params"]:
            self.state[p]["step"].fill_(float(gs["first"] - 1 + replays))
        if replays >= gs["steps"]:
            raise AcnError("FusedAdam: graph replays exceeded the precomputed Adam table; capture again")

    def _rows(self, bump: bool = True):
        """(p, grad, exp_avg, exp_avg_sq, kind) rows; kind indexes distinct (group, step) pairs.  bump:
        advance state['step'] first (torch increments it before the update)."""
        rows, kinds = [], []
        for gi, group in enumerate(self.param_groups):
            for p in group["params"]:
                if p.grad is None:
                    continue
                require_hip(p, "FusedAdam")
                if p.grad.is_sparse:
                    raise AcnError("FusedAdam: sparse gradients are not supported")
                st = self.state[p]
                if len(st) == 0:
                    st["step"] = torch.tensor(0.0, dtype=torch.float32)
                    st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                    st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                if bump:
                    st["step"] += 1
                key = (gi, int(st["step"].item()))
                if key not in kinds:
                    kinds.append(key)
                g = p.grad if p.grad.is_contiguous() else p.grad.contiguous()
                if not (p.is_contiguous() and st["exp_avg"].is_contiguous() and st["exp_avg_sq"].is_contiguous()):
                    raise AcnError("FusedAdam: parameters and state must be contiguous")
                if p.dtype != torch.float32 or g.dtype != torch.float32:
                    raise AcnError("FusedAdam: fp32 parameters/gradients only")
                rows.append((p, g, st["exp_avg"], st["exp_avg_sq"], kinds.index(key)))
        if len(kinds) > ACN_OPTIM_MAX_GROUPS:
            raise AcnError(f"FusedAdam: at most {ACN_OPTIM_MAX_GROUPS} distinct (group, step) pairs per step")
        return rows, kinds

    @torch.no_grad()
    def step(self, closure=None, max_norm: Optional[float] = None, sumsq_group=None):
        """One Adam step.  ``max_norm``: apply clip_grad_norm_(all params, max_norm) first (fused:
        the coefficient scales the gradients inside the update).  ``sumsq_group``: all-reduce the
        squared gradient norm over this process group before the coefficient (expert parallel)."""
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        rows, kinds = self._rows()
        if not rows:
            return loss
        device = rows[0][0].device
        key = tuple((p.data_ptr(), g.data_ptr(), m.data_ptr(), v.data_ptr(), k) for p, g, m, v, k in rows)
        if self._plan is None or self._plan.key != key:
            self._plan = _Plan(rows, device)
        plan = self._plan
        scale = None
        if max_norm is not None:
            distributed = sumsq_group is not None and dist.is_initialized() and dist.get_world_size(sumsq_group) > 1
            if distributed and self.shared_params:
                own = [r for r in rows if id(r[0]) not in self.shared_params]
                shr = [r for r in rows if id(r[0]) in self.shared_params]
                skey = (key, "split")
                if self._splans is None or self._splans[0] != skey:
                    self._splans = (skey, _Plan(own, device), _Plan(shr, device))
                total = grad_sumsq(None, device, self._splans[1])
                dist.all_reduce(total, group=sumsq_group)
                total = total + grad_sumsq(None, device, self._splans[2])
            else:
                total = grad_sumsq(None, device, plan)
                if distributed:
                    dist.all_reduce(total, group=sumsq_group)
            scale = clip_coef(total, max_norm)
            self.last_norm = scale
        if self._graph is not None:
            gs = self._graph
            if len(kinds) != len(self.param_groups) or any(k != (i, gs["first"]) for i, k in enumerate(kinds)):
                raise AcnError("FusedAdam graph mode: every parameter group needs gradients, all at the step "
                               f"after graph_begin ({gs['first']}); got {kinds}")
            gs["params"] = [r[0] for r in rows]
            check(_lib.lib().acn_adam_step_table(plan.descs.data_ptr(), plan.chunk_tensor.data_ptr(), plan.nchunks,
                                                 gs["table"].data_ptr(), len(self.param_groups),
                                                 gs["step_dev"].data_ptr(), gs["first"], gs["steps"],
                                                 None if scale is None else scale.data_ptr(), _stream(device)),
                  "acn_adam_step_table")
            bump_versions(gs["params"])
            return loss
        groups = (acn_adam_group * len(kinds))()
        for i, (gi, step) in enumerate(kinds):
            g = self.param_groups[gi]
            b1, b2 = g["betas"]
            groups[i] = acn_adam_group(float(g["lr"]), float(b1), float(b2), float(g["eps"]),
                                       float(g["weight_decay"]), int(step), 0)
        hook = EVENT_HOOK
        if hook is not None:
            e0 = torch.cuda.Event(enable_timing=True)
            e0.record()
        check(_lib.lib().acn_adam_step(plan.descs.data_ptr(), plan.chunk_tensor.data_ptr(), plan.nchunks, groups,
                                       len(kinds), None if scale is None else scale.data_ptr(), _stream(device)),
              "acn_adam_step")
        bump_versions([r[0] for r in rows])
        if hook is not None:
            e1 = torch.cuda.Event(enable_timing=True)
            e1.record()
            hook.append((e0, e1))
        return loss


class AmpScaler:
    """torch.cuda.amp.GradScaler for the fused training steps (use_amp: runtime_adapt.py:237-268,
    meta_core.py:123-136, trainer.py:24), its state on the device so a captured step replays it: ``scale``
    (float32[1]), ``tracker`` (int32[1]) and ``found`` (float32[1]).  The step multiplies its loss gradient by
    the scale (scaler.scale), and SlottedAdam.step(amp=...) folds unscale_ + clip_grad_norm_ + the found_inf
    skip + update() into acn_amp_unscale_coef.  ``AmpScaler.wrap(grad_scaler)`` works on a torch GradScaler's
    own _scale / _growth_tracker tensors, so its get_scale() / state_dict() follow the replayed steps.
    Defaults are GradScaler's."""

    def __init__(self, device, init_scale: float = 2.0 ** 16, growth_factor: float = 2.0,
                 backoff_factor: float = 0.5, growth_interval: int = 2000):
        self.growth_factor, self.backoff_factor = float(growth_factor), float(backoff_factor)
        self.growth_interval = int(growth_interval)
        self.scale_t = torch.full((1,), float(init_scale), device=device, dtype=torch.float32)
        self.tracker = torch.zeros(1, device=device, dtype=torch.int32)
        self.found = torch.zeros(1, device=device, dtype=torch.float32)
        self.torch_scaler = None

    @classmethod
    def wrap(cls, grad_scaler, device) -> "AmpScaler":
        """An AmpScaler on a torch.cuda.amp.GradScaler's device state (created lazily, as its scale() does)."""
        a = cls(device, grad_scaler.get_scale() if grad_scaler._scale is not None else grad_scaler._init_scale,
                grad_scaler.get_growth_factor(), grad_scaler.get_backoff_factor(), grad_scaler.get_growth_interval())
        if grad_scaler._scale is None:
            grad_scaler._lazy_init_scale_growth_tracker(device)
        if grad_scaler._scale.dtype != torch.float32 or grad_scaler._growth_tracker.dtype != torch.int32:
            raise AcnError("AmpScaler.wrap: unexpected GradScaler state dtypes")
        a.scale_t, a.tracker = grad_scaler._scale, grad_scaler._growth_tracker
        a.torch_scaler = grad_scaler
        return a

    @property
    def scale(self) -> torch.Tensor:
        """The current loss scale (device, 0-dim view)."""
        return self.scale_t.view(())

    def get_scale(self) -> float:
        return float(self.scale_t)

    def found_inf(self) -> bool:
        """Whether the last step was skipped for a non-finite gradient (host read)."""
        return bool(self.found[0] != 0)

    def state_dict(self) -> dict:
        """GradScaler.state_dict()'s keys."""
        return {"scale": self.get_scale(), "growth_factor": self.growth_factor, "backoff_factor": self.backoff_factor,
                "growth_interval": self.growth_interval,
                "_growth_tracker": int(self.tracker.reshape(-1)[0])}   # a wrapped GradScaler's tracker is 0-dim

    def reset(self, init_scale: float = 2.0 ** 16) -> None:
        """A fresh GradScaler's state (the reference builds one per runtime_adapt call, runtime_adapt.py:237)."""
        self.scale_t.fill_(float(init_scale))
        self.tracker.zero_()
        self.found.zero_()

    def load_state_dict(self, d: dict) -> None:
        self.growth_factor, self.backoff_factor = float(d["growth_factor"]), float(d["backoff_factor"])
        self.growth_interval = int(d["growth_interval"])
        self.scale_t.fill_(float(d["scale"]))
        self.tracker.fill_(int(d["_growth_tracker"]))

    def unscale_coef(self, total_sumsq: torch.Tensor, max_norm: Optional[float], out: torch.Tensor,
                     seg: Optional[torch.Tensor], K: int) -> None:
        from ._lib import ptr
        check(_lib.lib().acn_amp_unscale_coef(ptr(total_sumsq), float(max_norm or 0.0), ptr(self.scale_t),
                                              ptr(self.tracker), ptr(self.found), self.growth_factor,
                                              self.backoff_factor, self.growth_interval, ptr(out),
                                              ptr(seg) if seg is not None else None, int(K),
                                              _stream(out.device)), "acn_amp_unscale_coef")


ZERO_GRAD_FLAG = 1 << 16       # adam_step_slots: clear the gradient after reading it
NORM_ELSEWHERE_FLAG = 1 << 17  # grad_sumsq_slots_ex: this tensor's sum of squares comes from elsewhere


class SlottedAdam:
    """clip_grad_norm_ + torch.optim.Adam.step() of a FusedAdam's parameters with per-slot activity and
    step counters on the device, so a captured update replays correctly whichever slots a step reached.

    Every parameter belongs to a slot (``slot_of``: id(p) -> slot; slots 0..K-1 are experts, K.. are
    shared).  Expert slot k is active in a step iff ``seg[K + 1 + k] > 0`` on the device (the routed pair
    counts of routed.hip, or an activity vector written by the host); an inactive slot is skipped
    entirely -- no moment decay, no step increment -- which is what torch.optim.Adam does for a parameter
    whose .grad is None (runtime_adapt.py:305-309, meta_core.py:126-143).  Each slot has its own device
    step counter indexing a precomputed table of Adam constants (acn_adam_table_fill).  Gradients are the
    persistent buffers ``grads`` (id(p) -> tensor); ``flags`` adds ZERO_GRAD_FLAG / NORM_ELSEWHERE_FLAG bits
    per parameter.  Built outside any capture (plain host-to-device copies: the graph bakes in the
    addresses)."""

    def __init__(self, optimizer: FusedAdam, slot_of, grads, K: int, nslots: int, flags=None,
                 max_steps: int = 1 << 16, split_norm: bool = False, segmaps=None):
        L = _lib.lib()
        self.opt, self.K, self.nslots = optimizer, int(K), int(nslots)
        flags = flags or {}
        rows, fl, slots_seen = [], [], {}
        # torch creates a parameter's state at its first update: the moments of a parameter without state
        # are held here and enter optimizer.state once its slot has stepped (sync_state)
        self._pending = {}
        for gi, group in enumerate(optimizer.param_groups):
            for p in group["params"]:
                if id(p) not in slot_of:
                    continue  # parameters the step never differentiates
                st = optimizer.state.get(p)
                if not st:
                    st = self._pending[p] = {"step": torch.tensor(0.0, dtype=torch.float32),
                                             "exp_avg": torch.zeros_like(p), "exp_avg_sq": torch.zeros_like(p)}
                s = slot_of[id(p)]
                slots_seen[s] = max(slots_seen.get(s, 0), int(st["step"].item()))
                rows.append((p, grads[id(p)], st["exp_avg"], st["exp_avg_sq"], gi))
                fl.append(s | flags.get(id(p), 0))
        if not rows:
            raise AcnError("SlottedAdam: no parameter of the optimizer belongs to a slot")
        dev = rows[0][0].device
        self.device = dev
        self.rows = rows
        arr = (_lib.acn_param_desc * len(rows))()
        first = 0
        for t, (p, g, m, v, gi) in enumerate(rows):
            arr[t] = _lib.acn_param_desc(p.data_ptr(), g.data_ptr(), m.data_ptr(), v.data_ptr(), p.numel(), gi, first)
            first += (p.numel() + ACN_OPTIM_CHUNK - 1) // ACN_OPTIM_CHUNK
        self.nchunks = first
        self.descs = torch.frombuffer(bytearray(bytes(arr)), dtype=torch.uint8).to(dev)
        self.chunk_tensor = torch.cat([torch.full(((r[0].numel() + ACN_OPTIM_CHUNK - 1) // ACN_OPTIM_CHUNK,), t,
                                                  dtype=torch.int32) for t, r in enumerate(rows)]).to(dev)
        self.flags = torch.tensor(fl, device=dev, dtype=torch.int32)
        self._flags_host = list(fl)
        self.partials = torch.empty(first, device=dev, dtype=torch.float64)
        self.total = torch.empty(1, device=dev, dtype=torch.float64)
        self.scale = torch.ones(2, device=dev, dtype=torch.float32)
        self.ticket = torch.zeros(1, device=dev, dtype=torch.int32)   # acn_grad_clip_slots' counter
        self.step_dev = torch.tensor([slots_seen.get(s, 0) for s in range(self.nslots)], device=dev,
                                     dtype=torch.int32)
        self.ngroups = len(optimizer.param_groups)
        self.step0 = int(max(slots_seen.values(), default=0))
        self.table_steps = self.step0 + int(max_steps)
        self.table = torch.empty(int(L.acn_adam_table_bytes(self.ngroups, self.table_steps)), dtype=torch.uint8,
                                 device=dev)
        self._hparams = None
        self.refresh()
        # segment maps (acn_adam_step_slots_segmap): id(p) -> (now, ever) uint8 device maps of p's 64-B
        # segments; only for tensors whose group has weight_decay 0 (the skipped update is then exact)
        self.segmaps = None
        if segmaps:
            ptrs = []
            for (p, g, m, v, gi) in rows:
                mp = segmaps.get(id(p))
                ok = mp is not None and float(optimizer.param_groups[gi]["weight_decay"]) == 0.0 and p.numel() % 16 == 0
                ptrs += [mp[0].data_ptr(), mp[1].data_ptr()] if ok else [0, 0]
            if any(ptrs):
                self.segmaps = torch.tensor(ptrs, dtype=torch.int64).to(dev)
        # the clip norm's own pass visits only the tensors whose sum of squares it computes: rows flagged
        # NORM_ELSEWHERE (the routed step's tables: their share is telescoped from the scatter) would launch
        # one empty workgroup per 256 KiB chunk -- ~4,100 of them against ~120 live ones in C5 -- and the
        # reduction would then read ~4,100 partials (zeros) per step
        self.norm_plan = None
        keep = [t for t, f in enumerate(fl) if not f & NORM_ELSEWHERE_FLAG]
        if keep and len(keep) < len(rows):
            arr = (_lib.acn_param_desc * len(keep))()
            first = 0
            for j, t in enumerate(keep):
                p, g, m, v, gi = rows[t]
                arr[j] = _lib.acn_param_desc(p.data_ptr(), g.data_ptr(), m.data_ptr(), v.data_ptr(), p.numel(), gi,
                                             first)
                first += (p.numel() + ACN_OPTIM_CHUNK - 1) // ACN_OPTIM_CHUNK
            self.norm_plan = (torch.frombuffer(bytearray(bytes(arr)), dtype=torch.uint8).to(dev),
                              torch.cat([torch.full(((rows[t][0].numel() + ACN_OPTIM_CHUNK - 1) // ACN_OPTIM_CHUNK,),
                                                    j, dtype=torch.int32) for j, t in enumerate(keep)]).to(dev),
                              first, torch.tensor([fl[t] for t in keep], device=dev, dtype=torch.int32),
                              torch.empty(first, device=dev, dtype=torch.float64))
        # split_norm (expert parallel): the clip norm's sum of squares in two passes, the per-rank slots
        # (< K) first -- all-reduced over the group by the caller's function -- then the replicated shared
        # slots (>= K) once, added on top (the reference's clip_grad_norm_ over the whole container)
        self.split = bool(split_norm)
        if self.split:
            own_flags = [f | (NORM_ELSEWHERE_FLAG if (f & 0xffff) >= self.K else 0) for f in fl]
            self.flags_own = torch.tensor(own_flags, device=dev, dtype=torch.int32)
            sh = [(r, f) for r, f in zip(rows, fl) if (f & 0xffff) >= self.K]
            arr = (_lib.acn_param_desc * max(1, len(sh)))()
            first = 0
            for t, ((p, g, m, v, gi), f) in enumerate(sh):
                arr[t] = _lib.acn_param_desc(p.data_ptr(), g.data_ptr(), m.data_ptr(), v.data_ptr(), p.numel(), gi,
                                             first)
                first += (p.numel() + ACN_OPTIM_CHUNK - 1) // ACN_OPTIM_CHUNK
            if first == 0:
                raise AcnError("SlottedAdam(split_norm): no shared parameter")
            self.nchunks_sh = first
            self.descs_sh = torch.frombuffer(bytearray(bytes(arr)), dtype=torch.uint8).to(dev)
            self.chunk_sh = torch.cat([torch.full(((r[0].numel() + ACN_OPTIM_CHUNK - 1) // ACN_OPTIM_CHUNK,), t,
                                                  dtype=torch.int32) for t, (r, f) in enumerate(sh)]).to(dev)
            self.flags_sh = torch.tensor([f & ~NORM_ELSEWHERE_FLAG for r, f in sh], device=dev, dtype=torch.int32)
            self.partials_sh = torch.empty(first, device=dev, dtype=torch.float64)
            self.total_own = torch.empty(1, device=dev, dtype=torch.float64)

    def _group_hparams(self):
        return tuple((float(g["lr"]), tuple(float(b) for b in g["betas"]), float(g["eps"]), float(g["weight_decay"]))
                     for g in self.opt.param_groups)

    def refresh(self) -> None:
        """Re-fill the Adam constant table in place when a group's hyper-parameters changed (an LR
        scheduler); a captured graph keeps reading the same table.  Call outside capture, between steps."""
        hp = self._group_hparams()
        if hp == self._hparams:
            return
        L = _lib.lib()
        groups = (acn_adam_group * self.ngroups)()
        for i, (lr, (b1, b2), eps, wd) in enumerate(hp):
            groups[i] = acn_adam_group(lr, b1, b2, eps, wd, 1, 0)
        host = torch.empty(self.table.numel(), dtype=torch.uint8)
        check(L.acn_adam_table_fill(groups, self.ngroups, 1, self.table_steps, host.data_ptr(), host.numel()),
              "acn_adam_table_fill")
        self.table.copy_(host)
        self._hparams = hp

    def step_early(self, seg: torch.Tensor, hook=None) -> None:
        """Phase 1 of the split segment-mapped update (acn_adam_step_slots_segmap_phase): bump the active slots'
        step counters and update the table segments touched before but not this step (zero gradient: no clip
        coefficient needed), on the current stream (a side stream beside the step's forward / backward) -- as soon
        as the step's now[] marks exist.  step(..., phase=2) finishes the update after the clip coefficient."""
        if self.segmaps is None:
            raise AcnError("SlottedAdam.step_early needs segment maps")
        from ._lib import ptr
        s = _stream(self.device)
        if hook is not None:
            e0 = torch.cuda.Event(enable_timing=True)
            e0.record()
        check(_lib.lib().acn_adam_step_slots_segmap_phase(
            ptr(self.descs), ptr(self.chunk_tensor), self.nchunks, ptr(self.flags), ptr(self.table), self.ngroups,
            self.table_steps, ptr(self.step_dev), self.nslots, ptr(seg), self.K, None, ptr(self.segmaps), 1, s),
            "acn_adam_step_slots_segmap_phase")
        if hook is not None:
            e1 = torch.cuda.Event(enable_timing=True)
            e1.record()
            self._early_events = (e0, e1)

    def step(self, seg: torch.Tensor, max_norm: Optional[float], table_sumsq: Optional[torch.Tensor] = None,
             hook=None, allreduce=None, amp: Optional[AmpScaler] = None, phase: int = 0) -> None:
        """Clip norm over the active slots' gradients (+ ``table_sumsq``, a device double some kernel
        accumulated for NORM_ELSEWHERE tensors; reset by the norm pass), clip coefficient, then Adam over
        the active slots; per-slot step counters advance on the device.  ``allreduce`` (split_norm):
        in-place sum of a device double over the expert-parallel group, applied to the per-rank part.
        ``amp``: the gradients carry the AmpScaler's loss scale -- unscaled inside the Adam multiplier, the
        step skipped (seg[K] = -1) on a non-finite norm, the scale updated (GradScaler semantics)."""
        L = _lib.lib()
        s = _stream(self.device)
        from ._lib import ptr
        scale = None
        if max_norm is not None or amp is not None:
            if allreduce is not None:
                if not self.split:
                    raise AcnError("SlottedAdam.step(allreduce=...) needs split_norm=True")
                check(L.acn_grad_sumsq_slots_ex(ptr(self.descs), ptr(self.chunk_tensor), self.nchunks,
                                                ptr(self.flags_own), ptr(seg), self.K, ptr(self.partials),
                                                ptr(self.total_own), ptr(table_sumsq), s), "acn_grad_sumsq_slots_ex")
                allreduce(self.total_own)
                check(L.acn_grad_sumsq_slots_ex(ptr(self.descs_sh), ptr(self.chunk_sh), self.nchunks_sh,
                                                ptr(self.flags_sh), ptr(seg), self.K, ptr(self.partials_sh),
                                                ptr(self.total), ptr(self.total_own), s), "acn_grad_sumsq_slots_ex")
            else:
                descs, chunks, nch, flags, partials = self.norm_plan if self.norm_plan is not None else (
                    self.descs, self.chunk_tensor, self.nchunks, self.flags, self.partials)
                if amp is None and FUSED_CLIP:   # norm + clip coefficient in one launch
                    check(L.acn_grad_clip_slots(ptr(descs), ptr(chunks), nch, ptr(flags), ptr(seg), self.K,
                                                ptr(partials), ptr(self.total), ptr(table_sumsq), float(max_norm),
                                                ptr(self.scale), ptr(self.ticket), s), "acn_grad_clip_slots")
                else:
                    check(L.acn_grad_sumsq_slots_ex(ptr(descs), ptr(chunks), nch, ptr(flags), ptr(seg), self.K,
                                                    ptr(partials), ptr(self.total), ptr(table_sumsq), s),
                          "acn_grad_sumsq_slots_ex")
            if amp is not None:
                amp.unscale_coef(self.total, max_norm, self.scale, seg, self.K)
            elif allreduce is not None or not FUSED_CLIP:
                check(L.acn_clip_coef(ptr(self.total), float(max_norm), ptr(self.scale), s), "acn_clip_coef")
            scale = self.scale
        if hook is not None:
            e0 = torch.cuda.Event(enable_timing=True)
            e0.record()
        if self.segmaps is not None and phase == 2:    # after step_early: the segments touched now + dense tensors
            check(L.acn_adam_step_slots_segmap_phase(ptr(self.descs), ptr(self.chunk_tensor), self.nchunks,
                                                     ptr(self.flags), ptr(self.table), self.ngroups, self.table_steps,
                                                     ptr(self.step_dev), self.nslots, ptr(seg), self.K, ptr(scale),
                                                     ptr(self.segmaps), 2, s), "acn_adam_step_slots_segmap_phase")
        elif self.segmaps is not None:
            check(L.acn_adam_step_slots_segmap(ptr(self.descs), ptr(self.chunk_tensor), self.nchunks, ptr(self.flags),
                                               ptr(self.table), self.ngroups, self.table_steps, ptr(self.step_dev),
                                               self.nslots, ptr(seg), self.K, ptr(scale), ptr(self.segmaps), s),
                  "acn_adam_step_slots_segmap")
        else:
            check(L.acn_adam_step_slots(ptr(self.descs), ptr(self.chunk_tensor), self.nchunks, ptr(self.flags),
                                        ptr(self.table), self.ngroups, self.table_steps, ptr(self.step_dev),
                                        self.nslots, ptr(seg), self.K, ptr(scale), s), "acn_adam_step_slots")
        if hook is not None:
            e1 = torch.cuda.Event(enable_timing=True)
            e1.record()
            early = getattr(self, "_early_events", None) if phase == 2 else None
            self._early_events = None
            hook.append((e0, e1) if early is None else (early[0], early[1], e0, e1))   # pairs of events

    def sync_state(self, extra_slots=()) -> None:
        """Host state['step'] of every parameter from the per-slot device counters (state_dict, or before
        an eager FusedAdam step on the same optimizer).  A parameter enters optimizer.state once its slot
        has stepped, or when its slot is in ``extra_slots`` (about to step eagerly: the eager step then
        uses these moment tensors)."""
        steps = self.step_dev.cpu().tolist()
        if max(steps) > self.table_steps:
            raise AcnError("SlottedAdam: the Adam constant table is exhausted; build a new step object")
        for (p, g, m, v, gi), f in zip(self.rows, self._flags_host):
            slot = f & 0xffff
            if p in self._pending:
                if steps[slot] == 0 and slot not in extra_slots:
                    continue
                self.opt.state[p] = self._pending.pop(p)
            self.opt.state[p]["step"].fill_(float(steps[slot]))

    def load_state(self) -> int:
        """Per-slot device step counters from the optimizer's host state['step'] (after eager FusedAdam
        steps on the same optimizer, or a load_state_dict); returns the highest step.

        A captured step reads and writes the moment tensors it was built on (``rows``).  When an eager step
        or a load_state_dict gave a parameter other state tensors -- a pending parameter whose first update
        happened eagerly, or replaced tensors -- their values are copied into the row tensors and
        optimizer.state is pointed back at them, so the graph and the optimizer share one state."""
        steps = [0] * self.nslots
        for (p, g, m, v, gi), f in zip(self.rows, self._flags_host):
            st = self.opt.state.get(p)
            if st and p in self._pending:
                self._pending.pop(p)        # its first update ran eagerly: adopt that state below
            elif not st:
                st = self._pending[p]
            if st["exp_avg"] is not m:
                m.copy_(st["exp_avg"])
                st["exp_avg"] = m
            if st["exp_avg_sq"] is not v:
                v.copy_(st["exp_avg_sq"])
                st["exp_avg_sq"] = v
            n = int(st["step"].item())
            if n == 0 and self.opt.state.get(p) is st:
                self._pending[p] = self.opt.state.pop(p)   # never updated: no state entry, as in torch
            steps[f & 0xffff] = max(steps[f & 0xffff], n)
        if max(steps) + 1 > self.table_steps:
            raise AcnError("SlottedAdam: the Adam constant table is exhausted; build a new step object")
        self.step_dev.copy_(torch.tensor(steps, dtype=torch.int32))
        return max(steps)


def build_optimizer(P, model, fused: bool = True):
    """get_optimizer (common/utils.py:16-75) with FusedAdam for 'adam' (the online-stage config)."""
    base_lr = getattr(P, "lr", 1e-3)
    wd = getattr(P, "weight_decay", 0.0)
    groups = model.get_param_groups()
    pg = []
    for name, attr in (("encoding", "encoding_lr"), ("sigma", "sigma_lr"), ("color", "color_lr"),
                       ("background", "bg_lr")):
        if name in groups:
            lr = getattr(P, attr, None)
            pg.append({"params": list(groups[name]["params"]), "lr": float(base_lr if lr is None else lr), "name": name})
    opt = str(getattr(P, "optimizer", "adamw")).lower()
    if opt == "adam" and fused:
        return FusedAdam(pg, lr=base_lr, weight_decay=wd)
    if opt == "adam":
        return torch.optim.Adam(pg, lr=base_lr, weight_decay=wd)
    if opt == "adamw":
        return torch.optim.AdamW(pg, lr=base_lr, weight_decay=wd)
    if opt == "sgd":
        return torch.optim.SGD(pg, lr=base_lr, momentum=getattr(P, "momentum", 0.9), weight_decay=wd)
    raise ValueError(f"Unknown optimizer: {opt}")


def iter_params(model) -> Iterable[torch.nn.Parameter]:
    return [p for p in model.parameters() if p.requires_grad]
