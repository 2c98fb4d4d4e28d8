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
from ._lib import AcnError, acn_mlp, check, graph_capture, ptr
from .optim import NORM_ELSEWHERE_FLAG, ZERO_GRAD_FLAG, AmpScaler, FusedAdam, SlottedAdam, bump_versions
from .train import mse_color_loss

# Optional timing hook (bench.py): when set to a list, an eager step appends recorded HIP events
# bracketing the Adam launch (adam_step_slots) on the current stream.
EVENT_HOOK = None
# Same for the table-gradient scatter (hashgrid_bwd_pairs), the step's second-largest kernel.
BWD_HOOK = None

ALIGN = 128                # pair segment alignment = one MLP round (4 tiles x 32 slots)
# The tables' share of the clip norm from the scatter's returning atomics (acn_hashgrid_bwd_pairs_sumsq)
# instead of a pass over the K x 128 MiB gradient buffers
TELESCOPED_TABLE_NORM = os.environ.get("ACN_TELE_NORM", "1") != "0"
# The background head's forward / backward as two HIP launches (acn_background_fwd / _bwd) instead of the
# ~15 torch launches of its autograd graph
FUSED_BACKGROUND = os.environ.get("ACN_FUSED_BG", "1") != "0"
# Segment maps of the table gradients: the scatter marks the 64-B segments it adds into, and the Adam pass skips
# segments never touched (m = v = g = 0: bit-identical under torch's Adam with weight_decay 0) and reads no
# gradient for segments not touched this step
ADAM_SEGMAP = os.environ.get("ACN_ADAM_SEGMAP", "1") != "0"
# Split segment-mapped Adam: the early pass (segments touched before but not by this step) on a side stream
# beside the step's forward / backward, the late pass after the clip coefficient (the two passes
# contend for HBM with the step's own kernels: C5 1.75 -> 2.0 ms, so it stays off)
ADAM_EARLY = os.environ.get("ACN_ADAM_EARLY", "0") != "0"   # measured slower: off
# The background head's backward (two small launches) on a side stream beside the experts' backward chain
# (blend, MLP, table scatter), joined before the clip / Adam pass that reads its gradients
BG_SIDE = os.environ.get("ACN_BG_SIDE", "0") != "0"   # measured within noise: off
# The compositing glue of the step in one launch (acn_routed_composite_mse_train: blend, background forward,
# compositing, the linear MSE and the backward of all three down to the pair outputs) instead of eight launches
# and a copy; same arithmetic for every gradient (per-element; tests/test_routed_glue.py compares them bitwise).  The
# loss is a double sum whose order differs (per ray per workgroup here, element-strided in mse_linear_fwd_ws): it is
# equal after the float cast at the tested sizes, not by construction
FUSED_COMPOSITE = os.environ.get("ACN_FUSED_COMPOSITE", "1") != "0"


def draw_jitter(n: int, S: int, device) -> torch.Tensor:
    """The training jitter of one step: stratified_t_vals' rand_like of the (n, S) t grid
    (nerfs/ray_rendering.py:262-287), graph-safe philox under capture."""
    return torch.rand(n, S, device=device)


# the jitter source of jitter='draw' steps (tests substitute a recorded stream)
JITTER = draw_jitter


def _stream(device) -> int:
    return int(torch.cuda.current_stream(device).cuda_stream)


class RoutedAdaptStep:
    """One runtime_adapt update of a MetaContainer (routed, no active_module) per call.

    ``graph=True``: the first ``warmup`` calls run eagerly -- real updates on the caller's real batches --
    and the step is then captured once (the capture itself runs nothing) and replayed for every later
    full batch of ``n_rays`` rays.  A smaller batch (a loader's ragged last batch) runs eagerly through the
    same buffers.  ``jitter='draw'`` draws the training jitter inside the step like the reference, a
    caller-supplied (n, S) tensor per call otherwise (``jitter='given'``, for fixture replays)."""

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
        self.mlp_precision = ops.TRAIN_MLP_PRECISION   # training MLP kernels (ops.set_train_mlp_precision)
        # use_amp (ops.set_train_mlp_precision("amp")): the autocast(fp16) MLP arithmetic plus GradScaler --
        # the loss gradient enters the backward multiplied by the device loss scale, Adam unscales / skips
        self.amp = AmpScaler(model.submodules[0].xyz_encoder.hash_table.device) if self.mlp_precision == "amp" else None
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
        self.mws = torch.empty(int(ops.mlp_fn("acn_mlp_pairs_workspace_bytes", self.mlp_precision)(K)), device=dev,
                               dtype=torch.uint8)
        self.dw = torch.zeros(K, ops.MLP_DW_FLOATS, **f32)
        self.loss = torch.zeros((), **f32)
        self._one = torch.ones((), **f32)          # dL/dL of the explicit loss backward
        # ---- persistent gradients (every parameter's .grad is one of these buffers)
        self.gtables = [torch.zeros_like(e.hash_table) for e in encs]
        self.bg_params = list(model.bg_mlp.parameters())
        self.gbg = [torch.zeros_like(p) for p in self.bg_params]
        self.dirs = torch.zeros(N, 3, **f32)
        self.rgb = torch.zeros(N, 3, **f32)
        self.g_bg = torch.zeros(N, 3, **f32)
        self.gout = torch.zeros(cap, 4, **f32)
        self.cws = torch.zeros(int(L.acn_composite_mse_train_workspace_bytes()), device=dev, dtype=torch.uint8)
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
        # ---- slotted clip + Adam over every parameter of the optimizer's groups (optim.SlottedAdam)
        grads = {id(p): p.grad for p in model.parameters() if id(p) in slot_of}
        flags = {}
        for i in zero_of:
            flags[i] = (ZERO_GRAD_FLAG if self.clear_in_adam else 0) | (NORM_ELSEWHERE_FLAG if self.tele else 0)
        # segment maps: (K, 2, segments) bytes -- [k, 0] touched this step, [k, 1] touched before.  A table whose
        # moments may already be non-zero (optimizer state from earlier steps) starts all "touched before".
        self.segmaps = None
        smap = {}
        if ADAM_SEGMAP:
            nseg = encs[0].hash_table.numel() // 16
            self.segmaps = torch.zeros(K, 2, nseg, device=dev, dtype=torch.uint8)
            for k, e in enumerate(encs):
                st = optimizer.state.get(e.hash_table)
                if st and float(st.get("step", 0)) > 0:
                    self.segmaps[k, 1].fill_(1)
                smap[id(e.hash_table)] = (self.segmaps[k, 0], self.segmaps[k, 1])
            self._segnow = (C.c_void_p * K)(*[self.segmaps[k, 0].data_ptr() for k in range(K)])
        self.adam = SlottedAdam(optimizer, slot_of, grads, K, K + 1, flags, max_steps=max_steps, segmaps=smap)
        self.rows, self.flags, self.step_dev = self.adam.rows, self.adam.flags, self.adam.step_dev
        self.nslots, self.table_steps, self._step0 = self.adam.nslots, self.adam.table_steps, self.adam.step0
        self.scale = self.adam.scale
        self.table_sumsq = torch.zeros(1, device=dev, dtype=torch.float64)  # reset by grad_sumsq_slots_ex
        # split Adam (ADAM_EARLY): the table segments a step does not touch but earlier steps did (~40-60% of the
        # segment-mapped bytes) are updated on a side stream while the step's forward / backward runs -- their
        # gradient is zero, so they need no clip coefficient; the late pass updates the touched segments and the
        # dense tensors.  Not with use_amp (a found_inf skip is decided after the backward).
        self.early = ADAM_EARLY and self.segmaps is not None and self.amp is None
        self.side = torch.cuda.Stream(dev) if (self.early or BG_SIDE) else None
        self.replays = 0          # graph replays
        self.steps_done = 0       # every update this object ran (eager and replayed): Adam table rows used
        self.graph = None
        self._params = [r[0] for r in self.rows]
        self._eager_left = max(1, int(warmup)) if graph else 0   # eager real steps before the capture

    def _capture(self) -> None:
        """Record the full-batch step into one HIP graph (nothing executes; the static buffers keep their
        contents)."""
        dev = self.device
        torch.cuda.synchronize(dev)
        g = torch.cuda.CUDAGraph()
        with graph_capture(g):
            self._step(self.N)
        torch.cuda.synchronize(dev)
        self.graph = g

    # ------------------------------------------------------------------------------------------
    def _step(self, n: Optional[int] = None) -> None:
        L = _lib.lib()
        dev, K, S = self.device, self.K, self.S
        N = self.N if n is None else int(n)
        M = N * S
        s = _stream(dev)
        if not self.clear_in_adam:
            for g in self.gtables:
                g.zero_()
        u, t = self.u[:N], self.t[:N]
        if self.jitter_mode == "draw":   # the reference's rand_like(low) draw
            if JITTER is draw_jitter:
                torch.rand(N, S, device=dev, out=u)   # straight into the step's buffer (no copy launch)
            else:
                u.copy_(JITTER(N, S, dev))
        check(L.acn_routed_count(ptr(self.rays), N, S, ptr(u), C.byref(self.routing), ALIGN, ptr(t),
                                 ptr(self.seg), ptr(self.rws), self.rws.numel(), s), "acn_routed_count")
        check(L.acn_routed_scatter(ptr(self.rays), N, S, K, ptr(t), ptr(self.seg), C.cast(self._mins, C.c_void_p),
                                   C.cast(self._exts, C.c_void_p), self._lo, self._hi, ALIGN, ptr(self.rws),
                                   ptr(self.pidx), ptr(self.pw), ptr(self.x01), ptr(self.sh), ptr(self.pmap),
                                   ptr(self.pk), s), "acn_routed_scatter")
        enc = self.model.submodules[0].xyz_encoder
        capturing = torch.cuda.is_current_stream_capturing()   # no timing events inside a capture
        det = torch.are_deterministic_algorithms_enabled()
        ev_early = ev_bg = None
        if self.early and not det:
            # fork: the step's now[] marks from its pair list, then Adam's early pass, on the side stream
            main = torch.cuda.current_stream(dev)
            ev0 = torch.cuda.Event()
            ev0.record(main)
            self.side.wait_event(ev0)
            with torch.cuda.stream(self.side):
                check(L.acn_hashgrid_pairs_mark(ptr(self.x01), ptr(self.pk), ptr(self.pidx), ptr(self.seg), K,
                                                self._res, len(enc._res_host), enc.log2_hashmap_size,
                                                enc._interp_code, self._segnow, int(self.side.cuda_stream)),
                      "acn_hashgrid_pairs_mark")
                self.adam.step_early(self.seg, hook=EVENT_HOOK if self.graph is None and not capturing else None)
                ev_early = torch.cuda.Event()
                ev_early.record(self.side)
        check(L.acn_hashgrid_fwd_pairs(ptr(self.x01), ptr(self.pk), ptr(self.seg), K, self._tables, self._res,
                                       len(enc._res_host), enc.log2_hashmap_size, enc._interp_code, ptr(self.h0), s),
              "acn_hashgrid_fwd_pairs")
        mfn = lambda name: ops.mlp_fn(name, self.mlp_precision)  # noqa: E731
        check(mfn("acn_mlp_pack_pairs")(self._mlp_ptrs, K, ptr(self.mws), s), "acn_mlp_pack_pairs")
        check(mfn("acn_mlp_train_fwd_pairs")(ptr(self.h0), ptr(self.sh), ptr(self.seg), K, ptr(self.mws), ptr(self.out), s),
              "acn_mlp_train_fwd_pairs")
        rays, rgbs, dirs = self.rays[:N], self.rgbs[:N], self.dirs[:N]
        linear = str(self.P.color_space).lower() == "linear"
        if FUSED_COMPOSITE and self.bg_spec is not None and linear and S <= 1024:   # S: the kernel's LDS rows
            check(L.acn_routed_composite_mse_train(
                ptr(rays), N, S, ptr(t), ptr(self.out), ptr(self.pw), ptr(self.pmap), K, ptr(self.pidx), self.cap,
                ptr(self.seg[K:K + 1]), C.byref(self.bg_spec), ptr(rgbs), ptr(self._one if self.amp is None
                                                                            else self.amp.scale),
                ptr(self.rgb), ptr(dirs), ptr(self.g_bg), ptr(self.gout), ptr(self.loss), ptr(self.cws),
                self.cws.numel(), s), "acn_routed_composite_mse_train")
            ev_bg = self._head_bwd(dirs, self.g_bg[:N])
            self._experts_bwd(self.gout, enc, det, capturing, ev_early, ev_bg)
            return
        rs = ops.routed_blend_fwd(self.out, self.pw, self.pmap[:M]).view(N, S, 4).requires_grad_(True)
        # the shared part: compositing, colour transform and MSE under torch autograd (HIP kernels); the
        # background head as its fused HIP forward and backward (writing the persistent .grad buffers), or
        # under autograd when the head is not the HIP-supported SH-4 MLP
        from .ray_rendering import volume_render
        if self.bg_spec is not None and linear:
            # the kernels autograd would run (compositing, the linear-space MSE and their backwards), called
            # directly: no ones-fill for the loss gradient, no autograd bookkeeping launches
            dirs.copy_(rays[:, 3:6])
            rs_ = rs.detach()
            bg = ops.background_fwd(dirs, self.bg_spec)
            rgb = ops.volume_render(rs_, t, bg)[0]
            loss = ops.mse_linear_fwd(rgb, rgbs, out=self.loss)
            g_rgb = ops.mse_linear_bwd(rgb, rgbs, self._one if self.amp is None else self.amp.scale)
            g_rs, g_bg = ops.volume_render_bwd(rs_, t, bg, 1.0, g_rgb, None, None, None)
            ev_bg = self._head_bwd(dirs, g_bg)
        elif self.bg_spec is not None:
            dirs.copy_(rays[:, 3:6])
            bg = ops.background_fwd(dirs, self.bg_spec).requires_grad_(True)
            with torch.enable_grad():
                rgb = volume_render(rs, t, bg_rgb=bg)[0]
                loss = mse_color_loss(rgb, rgbs, self.P.color_space)
                g_rs, g_bg = torch.autograd.grad(loss if self.amp is None else loss * self.amp.scale, [rs, bg])
            ops.background_bwd(dirs, self.bg_spec, g_bg, self.gbg)
        else:
            with torch.enable_grad():
                bg = self.model.background_color(rays[:, 3:6])
                rgb = volume_render(rs, t, bg_rgb=bg)[0]
                loss = mse_color_loss(rgb, rgbs, self.P.color_space)
                grads = torch.autograd.grad(loss if self.amp is None else loss * self.amp.scale, [rs] + self.bg_params)
            g_rs = grads[0]
            for g, buf in zip(grads[1:], self.gbg):
                buf.copy_(g)
        if loss is not self.loss:
            self.loss.copy_(loss.detach())
        gout = ops.routed_blend_bwd(g_rs.reshape(M, 4).contiguous(), self.pidx, self.pw, live=self.seg[K:K + 1])
        self._experts_bwd(gout, enc, det, capturing, ev_early, ev_bg)

    def _head_bwd(self, dirs: torch.Tensor, g_bg: torch.Tensor):
        """The background head's backward into its persistent .grad buffers; on the side stream (BG_SIDE)
        it returns the event the Adam pass joins."""
        if BG_SIDE and self.side is not None:
            # fork: the head's backward beside the experts' chain; joined before Adam (ev_bg)
            main = torch.cuda.current_stream(self.device)
            e_fork = torch.cuda.Event()
            e_fork.record(main)
            self.side.wait_event(e_fork)
            with torch.cuda.stream(self.side):
                ops.background_bwd(dirs, self.bg_spec, g_bg, self.gbg)
                ev_bg = torch.cuda.Event()
                ev_bg.record(self.side)
            g_bg.record_stream(self.side)
            return ev_bg
        ops.background_bwd(dirs, self.bg_spec, g_bg, self.gbg)
        return None

    def _experts_bwd(self, gout: torch.Tensor, enc, det: bool, capturing: bool, ev_early, ev_bg) -> None:
        """From dL/d(pair outputs): the experts' MLP [dW | db] and table gradients, then clip + Adam."""
        L = _lib.lib()
        dev, K = self.device, self.K
        s = _stream(dev)
        mfn = lambda name: ops.mlp_fn(name, self.mlp_precision)  # noqa: E731
        check(mfn("acn_mlp_train_bwd_dw_pairs")(ptr(self.h0), ptr(self.sh), ptr(self.out), ptr(gout), ptr(self.seg), K,
                                           ptr(self.mws), ptr(self.dw), ptr(self.gh0), s), "acn_mlp_train_bwd_dw_pairs")
        bhook = BWD_HOOK if self.graph is None and not capturing else None
        if bhook is not None:
            b0 = torch.cuda.Event(enable_timing=True)
            b0.record()
        if det:
            self._table_bwd_deterministic(enc)
            if self.segmaps is not None:   # the sort-based backward marks no segments: the marks on their own
                check(L.acn_hashgrid_pairs_mark(ptr(self.x01), ptr(self.pk), ptr(self.pidx), ptr(self.seg), K,
                                                self._res, len(enc._res_host), enc.log2_hashmap_size,
                                                enc._interp_code, self._segnow, s), "acn_hashgrid_pairs_mark")
                if self.early:   # the same two passes, in sequence
                    self.adam.step_early(self.seg, hook=EVENT_HOOK if self.graph is None and not capturing else None)
        else:
            # the marks came from the side stream (early) or come with the scatter
            check(L.acn_hashgrid_bwd_pairs_segmap(ptr(self.x01), ptr(self.pk), ptr(self.pidx), ptr(self.seg), K,
                                                  ptr(self.gh0), self._gtables, self._res, len(enc._res_host),
                                                  enc.log2_hashmap_size, enc._interp_code,
                                                  ptr(self.table_sumsq) if self.tele else None,
                                                  self._segnow if self.segmaps is not None and not self.early
                                                  else None, s),
                  "acn_hashgrid_bwd_pairs_segmap")
        if bhook is not None:
            b1 = torch.cuda.Event(enable_timing=True)
            b1.record()
            bhook.append((b0, b1))
        if ev_early is not None:
            torch.cuda.current_stream(dev).wait_event(ev_early)   # join
        if ev_bg is not None:
            torch.cuda.current_stream(dev).wait_event(ev_bg)      # join: the head's gradients
        self.adam.step(self.seg, self.grad_clip, self.table_sumsq if self.tele else None,
                       hook=EVENT_HOOK if self.graph is None and not capturing else None, amp=self.amp,
                       phase=2 if self.early else 0)

    def _table_bwd_deterministic(self, enc) -> None:
        """Under torch.use_deterministic_algorithms(True): every expert's table gradient by the sort-based
        backward over its live pairs (acn_hashgrid_bwd_det: each row the serial fp32 sum of its contributions
        in pair order = sample order, bitwise reproducible) instead of float atomics, and the tables' share of
        the clip norm by a deterministic double reduction.  Reads the segment table to the host: eager only
        (a graph-replayed step runs this eagerly instead, __call__)."""
        if torch.cuda.is_current_stream_capturing():
            raise AcnError("RoutedAdaptStep: deterministic mode cannot be captured (it reads the pair counts)")
        K = self.K
        seg = self.seg.cpu().tolist()
        for k in range(K):
            s0, n = int(seg[k]), int(seg[K + 1 + k])
            if n:
                ops.hashgrid_bwd(self.x01[s0:s0 + n], self.gh0[s0:s0 + n], enc._res_host, enc.log2_hashmap_size, 2,
                                 enc._interp_code, deterministic=True, out=self.gtables[k])
        if self.tele:
            tot = torch.zeros((), device=self.device, dtype=torch.float64)
            for g in self.gtables:
                tot = tot + (g.double() ** 2).sum()
            self.table_sumsq.copy_(tot.view(1))

    def __call__(self, rays: torch.Tensor, rgbs: torch.Tensor, jitter_u: Optional[torch.Tensor] = None) -> torch.Tensor:
        n = int(rays.shape[0])
        if rays.dim() != 2 or rays.shape[1] != 8 or tuple(rgbs.shape) != (n, 3) or not 0 < n <= self.N:
            raise AcnError(f"RoutedAdaptStep was built for batches of up to {self.N} rays; got {tuple(rays.shape)}, "
                           f"{tuple(rgbs.shape)}")
        # every update, eager or replayed, consumes one row of the Adam constant table (per-slot device
        # counters never run ahead of the number of updates)
        if self._step0 + self.steps_done + 1 > self.table_steps:
            raise AcnError("RoutedAdaptStep: the Adam constant table is exhausted; build a new step object")
        self.rays[:n].copy_(rays, non_blocking=True)
        self.rgbs[:n].copy_(rgbs, non_blocking=True)
        if self.jitter_mode == "given":
            if jitter_u is None or tuple(jitter_u.shape) != (n, self.S):
                raise AcnError(f"RoutedAdaptStep(jitter='given') needs jitter_u of shape ({n}, {self.S}) per call")
            self.u[:n].copy_(jitter_u, non_blocking=True)
        det = torch.are_deterministic_algorithms_enabled()   # eager: the deterministic table backward
        if n == self.N and self.graph is not None and not det:
            self.graph.replay()
            self.replays += 1
        else:
            self._step(n)
            if n == self.N and self._eager_left > 0 and not det:
                self._eager_left -= 1
                if self._eager_left == 0:
                    self._capture()
        self.steps_done += 1
        bump_versions(self._params)  # the kernels wrote them: packed render images are stale
        return self.loss

    @property
    def last_norm(self) -> torch.Tensor:
        """(total_norm, clip coefficient) of the last step (device), as FusedAdam.last_norm."""
        return self.scale

    def segment_stats(self):
        """(segments touched by the last step's scatter, segments ever updated, segments in all tables), from
        the maps after a step (the last step's marks are in 'ever' once its Adam pass ran).  Host read."""
        if self.segmaps is None:
            return None
        ever = int(self.segmaps[:, 1].sum())
        return ever, int(self.segmaps[:, 1].numel())

    def segment_line_stats(self):
        """128-B lines (two adjacent 64-B segments) of the tables holding at least one ever-updated segment:
        what the segment-mapped Adam's reads fetch if HBM lines are filled whole.  Host read."""
        if self.segmaps is None:
            return None
        ev = self.segmaps[:, 1]
        pairs = ev[:, : ev.shape[1] // 2 * 2].reshape(ev.shape[0], -1, 2)
        return int((pairs.amax(dim=2) != 0).sum())

    def sync_state(self) -> None:
        """Host state['step'] of every parameter from the per-slot device counters (state_dict, or before
        an eager FusedAdam step on the same optimizer)."""
        self.adam.sync_state()

    def load_state(self) -> None:
        """Per-slot device step counters from the optimizer's host state['step'] (after eager FusedAdam
        steps taken on the same optimizer outside this object), and the Adam constants from the current
        group hyper-parameters."""
        before = self.adam.step_dev.cpu().tolist()
        top = self.adam.load_state()
        self.adam.refresh()
        if self.segmaps is not None:
            # an eager step on slot k (runtime_adapt(active_module=k), or the eager routed step) may have moved
            # any row of table k: every segment of a table whose slot counter changed counts as touched, so the
            # segment-mapped Adam keeps decaying its moments
            after = self.adam.step_dev.cpu().tolist()
            for k in range(self.K):
                if after[k] != before[k]:
                    self.segmaps[k, 1].fill_(1)
        self._step0 = top - self.steps_done   # keeps the exhaustion guard exact
