"""runtime_adapt's update of the ROUTED container on the pair kernels, capturable as one HIP graph.

Reference: pipelines/online_stage/runtime_adapt.py:286-309 with ``active_module=None`` -- the online
stage adapts the whole soft-routed container (models/inr/meta_container.py:275-343): every expert a
sample is routed to renders it, the blend is a weighted index_add_ in expert order, gradients reach
exactly the experts that received samples (the others keep grad None and Adam skips them), then
clip_grad_norm_(1.0) and Adam over every parameter with a gradient.

Here one step is a fixed sequence of launches with no host synchronisation, so it replays as a graph:

    routed_count / routed_scatter   t, routing weights, (sample, expert) pair slots, segments padded
                                    to 128 (routed.hip); jitter = torch.rand(N, S) (the reference's
                                    rand_like draw, graph-safe philox)
    hashgrid_fwd_pairs              h0 of every slot through its expert's table
    mlp_pack_pairs + fwd_pairs      the K expert MLPs on MFMA, per slot
    routed_blend_fwd                (M, 4) = sum_k y_k w_k in expert order
    background + volume_render + MSE under torch autograd (the small shared part)
    routed_blend_bwd / mlp_bwd_dw_pairs / hashgrid_bwd_pairs
                                    per-expert [dW | db] (deterministic order) and table gradients
                                    (float atomics into persistent buffers)
    grad_sumsq_slots + clip_coef + adam_step_slots
                                    clip norm and Adam over the ACTIVE experts only (pair count > 0,
                                    decided on the device) + the shared background head; the table
                                    gradients are cleared by the Adam pass itself.

Buffers are sized for the worst case (every sample routed to every expert), so the step never needs
the pair count on the host.  Parameters keep torch's optimizer state layout: exp_avg / exp_avg_sq are
the FusedAdam state tensors, state['step'] is synchronised from the per-expert device counters.
"""
from __future__ import annotations

import ctypes as C
import os
from typing import Optional

import numpy as np
import torch

from . import _lib, ops
from ._lib import ACN_OPTIM_CHUNK, AcnError, acn_adam_group, acn_mlp, check, ptr
from .optim import FusedAdam, bump_versions
from .train import mse_color_loss

# Optional timing hook (bench.py): when set to a list, an eager step appends recorded HIP events
# bracketing the Adam launch (adam_step_slots) on the current stream.
EVENT_HOOK = None
# Same for the table-gradient scatter (hashgrid_bwd_pairs), the step's second-largest kernel.
BWD_HOOK = None

ALIGN = 128                # pair segment alignment = one MLP round (4 tiles x 32 slots)
ZERO_GRAD_FLAG = 1 << 16   # adam_step_slots: clear the gradient after reading it
NORM_ELSEWHERE_FLAG = 1 << 17  # grad_sumsq_slots_ex: this tensor's sum of squares comes from the table scatter
# The tables' share of the clip norm from the scatter's returning atomics (acn_hashgrid_bwd_pairs_sumsq)
# instead of a pass over the K x 128 MiB gradient buffers
TELESCOPED_TABLE_NORM = os.environ.get("ACN_TELE_NORM", "1") != "0"
# The background head's forward / backward as two HIP launches (acn_background_fwd / _bwd) instead of the
# ~15 torch launches of its autograd graph
FUSED_BACKGROUND = os.environ.get("ACN_FUSED_BG", "1") != "0"


def _stream(device) -> int:
    return int(torch.cuda.current_stream(device).cuda_stream)


class RoutedAdaptStep:
    """One runtime_adapt update of a MetaContainer (routed, no active_module) per call.

    ``graph=True`` captures the step once (after ``warmup`` eager steps, which are real updates) and
    replays it; ``jitter='draw'`` draws the training jitter inside the step like the reference, a
    caller-supplied (N, S) tensor per call otherwise (``jitter='given'``, for fixture replays)."""

    def __init__(self, P, model, n_rays: int, optimizer: FusedAdam, grad_clip: Optional[float] = 1.0,
                 graph: bool = True, warmup: int = 1, max_steps: int = 1 << 16, jitter: str = "draw",
                 clear_in_adam: bool = True):
        from .meta_container import MetaContainer
        if not isinstance(model, MetaContainer) or not all(s._fusable for s in model.submodules):
            raise AcnError("RoutedAdaptStep: a MetaContainer of reference-configuration experts is required")
        if not isinstance(optimizer, FusedAdam):
            raise AcnError("RoutedAdaptStep needs FusedAdam")
        if not model.use_bg_nerf:
            raise AcnError("RoutedAdaptStep: the background head is part of the reference configuration")
        encs = [s.xyz_encoder for s in model.submodules]
        e0 = encs[0]
        if any(e._res_host != e0._res_host or e.log2_hashmap_size != e0.log2_hashmap_size
               or e._interp_code != e0._interp_code for e in encs) or e0._interp_code == 0:
            raise AcnError("RoutedAdaptStep: experts must share one Linear/Smoothstep hash-grid configuration")
        self.P, self.model, self.opt = P, model, optimizer
        self.grad_clip = grad_clip
        self.jitter_mode = jitter
        # clear_in_adam=False keeps the gradients readable after the step (tests): the table gradients
        # are then zeroed at the start of the next step instead of by the Adam pass
        self.clear_in_adam = bool(clear_in_adam)
        self.tele = TELESCOPED_TABLE_NORM and grad_clip is not None
        dev = e0.hash_table.device
        self.device = dev
        K = len(model.submodules)
        S = int(P.ray_samples)
        N = int(n_rays)
        M = N * S
        cap = M * K + K * ALIGN
        self.K, self.N, self.S, self.M, self.cap = K, N, S, M, cap
        f32 = dict(device=dev, dtype=torch.float32)
        i32 = dict(device=dev, dtype=torch.int32)
        L = _lib.lib()
        # ---- static inputs / pair buffers
        self.rays = torch.zeros(N, 8, **f32)
        self.rgbs = torch.zeros(N, 3, **f32)
        self.u = torch.zeros(N, S, **f32)
        self.t = torch.empty(N, S, **f32)
        self.seg = torch.zeros(2 * K + 1, device=dev, dtype=torch.int64)
        self.rws = torch.empty(int(L.acn_routed_workspace_bytes(M, K)), device=dev, dtype=torch.uint8)
        self.pidx = torch.empty(cap, **i32)
        self.pw = torch.empty(cap, **f32)
        self.pk = torch.empty(cap, **i32)
        self.x01 = torch.empty(cap, 3, **f32)
        self.sh = torch.empty(cap, 16, **f32)
        self.pmap = torch.empty(M, K, **i32)
        self.h0 = torch.empty(cap, 32, **f32)
        self.out = torch.empty(cap, 4, **f32)
        self.gh0 = torch.empty(cap, 32, **f32)
        self.mws = torch.empty(int(L.acn_mlp_pairs_workspace_bytes(K)), device=dev, dtype=torch.uint8)
        self.dw = torch.zeros(K, ops.MLP_DW_FLOATS, **f32)
        self.loss = torch.zeros((), **f32)
        # ---- persistent gradients (every parameter's .grad is one of these buffers)
        self.gtables = [torch.zeros_like(e.hash_table) for e in encs]
        self.bg_params = list(model.bg_mlp.parameters())
        self.gbg = [torch.zeros_like(p) for p in self.bg_params]
        self.dirs = torch.zeros(N, 3, **f32)
        try:   # (acn_background, the tensors it points into)
            self.bg_spec, self._bg_keep = model.background_spec() if FUSED_BACKGROUND else (None, None)
        except AcnError:
            self.bg_spec, self._bg_keep = None, None
        slot_of, zero_of = {}, {}
        for k, sub in enumerate(model.submodules):
            sub.xyz_encoder.hash_table.grad = self.gtables[k]
            slot_of[id(sub.xyz_encoder.hash_table)] = k
            zero_of[id(sub.xyz_encoder.hash_table)] = True
            views, o = [], 0
            for shp in ops.MLP_DW_SHAPES:
                n = int(np.prod(shp))
                views.append(self.dw[k, o:o + n].view(shp))
                o += n
            for (name, t), g in zip(sub._mlp_tensors(None).items(), views):
                t.grad = g
                slot_of[id(t)] = k
        for p, g in zip(self.bg_params, self.gbg):
            p.grad = g
            slot_of[id(p)] = K
        self._mlp_structs = [ops._mlp_struct([t for t in s._mlp_tensors(None).values()]) for s in model.submodules]
        self._mlp_ptrs = (C.POINTER(acn_mlp) * K)(*[C.pointer(w) for w in self._mlp_structs])
        self._tables = (C.c_void_p * K)(*[e.hash_table.data_ptr() for e in encs])
        self._gtables = (C.c_void_p * K)(*[g.data_ptr() for g in self.gtables])
        self._res = (C.c_int32 * len(e0._res_host))(*e0._res_host)
        boxes = [s._host_box() for s in model.submodules]
        self._mins = (C.c_float * (3 * K))(*[float(v) for b in boxes for v in b[0]])
        self._exts = (C.c_float * (3 * K))(*[float(v) for b in boxes for v in b[1]])
        lo = np.float32(1e-6)
        self._lo, self._hi = C.c_float(lo), C.c_float(np.float32(1.0) - lo)
        self.routing = model.routing_spec()
        # ---- slotted optimizer plan over every parameter of the optimizer's groups
        rows, flags, slots_seen = [], [], {}
        for gi, group in enumerate(optimizer.param_groups):
            for p in group["params"]:
                if id(p) not in slot_of:
                    continue  # parameters the routed step never differentiates (none in the reference setup)
                st = optimizer.state[p]
                if len(st) == 0:
                    st["step"] = torch.tensor(0.0, dtype=torch.float32)
                    st["exp_avg"] = torch.zeros_like(p)
                    st["exp_avg_sq"] = torch.zeros_like(p)
                s = slot_of[id(p)]
                slots_seen.setdefault(s, int(st["step"].item()))
                rows.append((p, p.grad, st["exp_avg"], st["exp_avg_sq"], gi))
                fl = s | (ZERO_GRAD_FLAG if zero_of.get(id(p)) and self.clear_in_adam else 0)
                if zero_of.get(id(p)) and self.tele:
                    fl |= NORM_ELSEWHERE_FLAG
                flags.append(fl)
        self.rows = rows
        self.nslots = K + 1
        arr = (_lib.acn_param_desc * len(rows))()
        first = 0
        for t, (p, g, m, v, gi) in enumerate(rows):
            arr[t] = _lib.acn_param_desc(p.data_ptr(), g.data_ptr(), m.data_ptr(), v.data_ptr(), p.numel(), gi, first)
            first += (p.numel() + ACN_OPTIM_CHUNK - 1) // ACN_OPTIM_CHUNK
        self.nchunks = first
        # built outside any capture: plain host-to-device copies (the graph bakes in the device addresses)
        self.descs = torch.frombuffer(bytearray(bytes(arr)), dtype=torch.uint8).to(dev)
        self.chunk_tensor = torch.cat([torch.full(((r[0].numel() + ACN_OPTIM_CHUNK - 1) // ACN_OPTIM_CHUNK,), t,
                                                  dtype=torch.int32) for t, r in enumerate(rows)]).to(dev)
        self.flags = torch.tensor(flags, **i32)
        self.partials = torch.empty(first, device=dev, dtype=torch.float64)
        self.total = torch.empty(1, device=dev, dtype=torch.float64)
        self.table_sumsq = torch.zeros(1, device=dev, dtype=torch.float64)  # reset by grad_sumsq_slots_ex
        self.scale = torch.ones(2, **f32)
        self.step_dev = torch.tensor([slots_seen.get(s, 0) for s in range(self.nslots)], **i32)
        ng = len(optimizer.param_groups)
        self._step0 = int(max(slots_seen.values(), default=0))
        self.table_steps = self._step0 + int(max_steps)
        groups = (acn_adam_group * ng)()
        for i, g in enumerate(optimizer.param_groups):
            b1, b2 = g["betas"]
            groups[i] = acn_adam_group(float(g["lr"]), float(b1), float(b2), float(g["eps"]), float(g["weight_decay"]),
                                       1, 0)
        nbytes = int(L.acn_adam_table_bytes(ng, self.table_steps))
        host = torch.empty(nbytes, dtype=torch.uint8)
        check(L.acn_adam_table_fill(groups, ng, 1, self.table_steps, host.data_ptr(), nbytes), "acn_adam_table_fill")
        self.table = host.to(dev)
        self.ngroups = ng
        self.replays = 0
        self.graph = None
        self._params = [r[0] for r in rows]
        if graph:
            side = torch.cuda.Stream(dev)
            side.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(side):
                for _ in range(max(1, int(warmup))):
                    self._step()
            torch.cuda.current_stream(dev).wait_stream(side)
            torch.cuda.synchronize(dev)
            self.graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self.graph):
                self._step()

    # ------------------------------------------------------------------------------------------
    def _step(self) -> None:
        L = _lib.lib()
        dev, K, N, S, M = self.device, self.K, self.N, self.S, self.M
        s = _stream(dev)
        if not self.clear_in_adam:
            for g in self.gtables:
                g.zero_()
        if self.jitter_mode == "draw":
            self.u.copy_(torch.rand(N, S, device=dev))  # the reference's rand_like(low) draw
        check(L.acn_routed_count(ptr(self.rays), N, S, ptr(self.u), C.byref(self.routing), ALIGN, ptr(self.t),
                                 ptr(self.seg), ptr(self.rws), self.rws.numel(), s), "acn_routed_count")
        check(L.acn_routed_scatter(ptr(self.rays), N, S, K, ptr(self.t), ptr(self.seg), C.cast(self._mins, C.c_void_p),
                                   C.cast(self._exts, C.c_void_p), self._lo, self._hi, ALIGN, ptr(self.rws),
                                   ptr(self.pidx), ptr(self.pw), ptr(self.x01), ptr(self.sh), ptr(self.pmap),
                                   ptr(self.pk), s), "acn_routed_scatter")
        enc = self.model.submodules[0].xyz_encoder
        check(L.acn_hashgrid_fwd_pairs(ptr(self.x01), ptr(self.pk), ptr(self.seg), K, self._tables, self._res,
                                       len(enc._res_host), enc.log2_hashmap_size, enc._interp_code, ptr(self.h0), s),
              "acn_hashgrid_fwd_pairs")
        check(L.acn_mlp_pack_pairs(self._mlp_ptrs, K, ptr(self.mws), s), "acn_mlp_pack_pairs")
        check(L.acn_mlp_train_fwd_pairs(ptr(self.h0), ptr(self.sh), ptr(self.seg), K, ptr(self.mws), ptr(self.out), s),
              "acn_mlp_train_fwd_pairs")
        rs = ops.routed_blend_fwd(self.out, self.pw, self.pmap).view(N, S, 4).requires_grad_(True)
        # the shared part: compositing, colour transform and MSE under torch autograd (HIP kernels); the
        # background head as its fused HIP forward and backward (writing the persistent .grad buffers), or
        # under autograd when the head is not the HIP-supported SH-4 MLP
        from .ray_rendering import volume_render
        if self.bg_spec is not None:
            self.dirs.copy_(self.rays[:, 3:6])
            bg = ops.background_fwd(self.dirs, self.bg_spec).requires_grad_(True)
            with torch.enable_grad():
                rgb = volume_render(rs, self.t, bg_rgb=bg)[0]
                loss = mse_color_loss(rgb, self.rgbs, self.P.color_space)
                g_rs, g_bg = torch.autograd.grad(loss, [rs, bg])
            ops.background_bwd(self.dirs, self.bg_spec, g_bg, self.gbg)
        else:
            with torch.enable_grad():
                bg = self.model.background_color(self.rays[:, 3:6])
                rgb = volume_render(rs, self.t, bg_rgb=bg)[0]
                loss = mse_color_loss(rgb, self.rgbs, self.P.color_space)
                grads = torch.autograd.grad(loss, [rs] + self.bg_params)
            g_rs = grads[0]
            for g, buf in zip(grads[1:], self.gbg):
                buf.copy_(g)
        self.loss.copy_(loss.detach())
        gout = ops.routed_blend_bwd(g_rs.reshape(M, 4).contiguous(), self.pidx, self.pw, live=self.seg[K:K + 1])
        check(L.acn_mlp_train_bwd_dw_pairs(ptr(self.h0), ptr(self.sh), ptr(self.out), ptr(gout), ptr(self.seg), K,
                                           ptr(self.mws), ptr(self.dw), ptr(self.gh0), s), "acn_mlp_train_bwd_dw_pairs")
        bhook = BWD_HOOK if self.graph is None else None
        if bhook is not None:
            b0 = torch.cuda.Event(enable_timing=True)
            b0.record()
        check(L.acn_hashgrid_bwd_pairs_sumsq(ptr(self.x01), ptr(self.pk), ptr(self.pidx), ptr(self.seg), K,
                                             ptr(self.gh0), self._gtables, self._res, len(enc._res_host),
                                             enc.log2_hashmap_size, enc._interp_code,
                                             ptr(self.table_sumsq) if self.tele else None, s),
              "acn_hashgrid_bwd_pairs_sumsq")
        if bhook is not None:
            b1 = torch.cuda.Event(enable_timing=True)
            b1.record()
            bhook.append((b0, b1))
        scale = None
        if self.grad_clip is not None:
            check(L.acn_grad_sumsq_slots_ex(ptr(self.descs), ptr(self.chunk_tensor), self.nchunks, ptr(self.flags),
                                            ptr(self.seg), K, ptr(self.partials), ptr(self.total),
                                            ptr(self.table_sumsq) if self.tele else None, s),
                  "acn_grad_sumsq_slots_ex")
            check(L.acn_clip_coef(ptr(self.total), float(self.grad_clip), ptr(self.scale), s), "acn_clip_coef")
            scale = self.scale
        hook = EVENT_HOOK if self.graph is None else None
        if hook is not None:
            e0 = torch.cuda.Event(enable_timing=True)
            e0.record()
        check(L.acn_adam_step_slots(ptr(self.descs), ptr(self.chunk_tensor), self.nchunks, ptr(self.flags),
                                    ptr(self.table), self.ngroups, self.table_steps, ptr(self.step_dev), self.nslots,
                                    ptr(self.seg), K, ptr(scale), s), "acn_adam_step_slots")
        if hook is not None:
            e1 = torch.cuda.Event(enable_timing=True)
            e1.record()
            hook.append((e0, e1))

    def __call__(self, rays: torch.Tensor, rgbs: torch.Tensor, jitter_u: Optional[torch.Tensor] = None) -> torch.Tensor:
        if tuple(rays.shape) != (self.N, 8) or tuple(rgbs.shape) != (self.N, 3):
            raise AcnError(f"RoutedAdaptStep was built for {self.N} rays; got {tuple(rays.shape)}, {tuple(rgbs.shape)}")
        if self._step0 + self.replays + 1 > self.table_steps:
            raise AcnError("RoutedAdaptStep: the Adam constant table is exhausted; build a new step object")
        self.rays.copy_(rays, non_blocking=True)
        self.rgbs.copy_(rgbs, non_blocking=True)
        if self.jitter_mode == "given":
            if jitter_u is None:
                raise AcnError("RoutedAdaptStep(jitter='given') needs jitter_u per call")
            self.u.copy_(jitter_u, non_blocking=True)
        if self.graph is not None:
            self.graph.replay()
        else:
            self._step()
        self.replays += 1
        bump_versions(self._params)  # the kernels wrote them: packed render images are stale
        return self.loss

    @property
    def last_norm(self) -> torch.Tensor:
        """(total_norm, clip coefficient) of the last step (device), as FusedAdam.last_norm."""
        return self.scale

    def sync_state(self) -> None:
        """Host state['step'] of every parameter from the per-slot device counters (state_dict)."""
        steps = self.step_dev.cpu().tolist()
        if max(steps) >= self.table_steps:
            raise AcnError("RoutedAdaptStep: the Adam constant table is exhausted; build a new step object")
        for (p, g, m, v, gi), f in zip(self.rows, self.flags.cpu().tolist()):
            self.opt.state[p]["step"].fill_(float(steps[f & 0xffff]))
