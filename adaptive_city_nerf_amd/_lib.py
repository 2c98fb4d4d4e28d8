"""ctypes binding of libacnerf.so (the C ABI declared in include/acnerf.h).

This is the Python-side FFI stub of the drop-in boundary: every call passes raw device pointers
of torch tensors (owned by PyTorch's caching allocator) plus the current HIP stream.  There is no
CPU fallback: if the library or a HIP device is missing, calls raise.
"""
from __future__ import annotations

import contextlib
import ctypes as C
import os
import threading
from pathlib import Path

import torch  # must be imported before the library: libacnerf.so binds torch's libamdhip64.so.7

PKG = Path(__file__).resolve().parent
LIB_PATH = Path(os.environ.get("ACNERF_LIB", PKG / "libacnerf.so"))

ACN_MAX_LEVELS = 32
ACN_MAX_EXPERTS = 16
ACN_BG_NONE, ACN_BG_CONST, ACN_BG_MLP = 0, 1, 2
INTERP = {"Nearest": 0, "Linear": 1, "Smoothstep": 2}


class AcnError(RuntimeError):
    pass


class acn_expert(C.Structure):
    _fields_ = [
        ("table", C.c_void_p),
        ("L", C.c_int32), ("log2T", C.c_int32), ("F", C.c_int32), ("interp", C.c_int32),
        ("res", C.c_int32 * ACN_MAX_LEVELS),
        ("aabb_min", C.c_float * 3), ("aabb_extent", C.c_float * 3),
        ("sig_w0", C.c_void_p), ("sig_b0", C.c_void_p),
        ("sig_w1", C.c_void_p), ("sig_b1", C.c_void_p),
        ("sigh_w", C.c_void_p), ("sigh_b", C.c_void_p),
        ("geo_w", C.c_void_p), ("geo_b", C.c_void_p),
        ("col_w0", C.c_void_p), ("col_b0", C.c_void_p),
        ("col_w1", C.c_void_p), ("col_b1", C.c_void_p),
        ("col_w2", C.c_void_p), ("col_b2", C.c_void_p),
    ]


class acn_routing(C.Structure):
    _fields_ = [("K", C.c_int32), ("cluster_2d", C.c_int32), ("boundary_margin", C.c_float),
                ("centroids", (C.c_float * 3) * ACN_MAX_EXPERTS)]


class acn_background(C.Structure):
    _fields_ = [("mode", C.c_int32), ("hidden", C.c_int32), ("color", C.c_float * 3),
                ("w1", C.c_void_p), ("b1", C.c_void_p), ("w2", C.c_void_p), ("b2", C.c_void_p)]


ACN_OPTIM_CHUNK = 65536
ACN_OPTIM_MAX_GROUPS = 8


class acn_param_desc(C.Structure):
    _fields_ = [("param", C.c_void_p), ("grad", C.c_void_p), ("exp_avg", C.c_void_p), ("exp_avg_sq", C.c_void_p),
                ("numel", C.c_int64), ("group", C.c_int32), ("first_chunk", C.c_int32)]


class acn_mlp(C.Structure):
    _fields_ = [(n, C.c_void_p) for n in ("w0", "b0", "w1", "b1", "wsh", "bsh", "wg", "bg", "wc0", "bc0", "wc1",
                                          "bc1", "wc2", "bc2")]


class acn_adam_group(C.Structure):
    _fields_ = [("lr", C.c_double), ("beta1", C.c_double), ("beta2", C.c_double), ("eps", C.c_double),
                ("weight_decay", C.c_double), ("step", C.c_int32), ("pad", C.c_int32)]


_lib = None
_lock = threading.Lock()
vp, i64, i32, f32, sz = C.c_void_p, C.c_int64, C.c_int, C.c_float, C.c_size_t

SIGNATURES = {
    "acn_version": ([], C.c_int),
    "acn_last_error": ([C.c_char_p, sz], C.c_int),
    "acn_hashgrid_fwd": ([vp, i64, vp, vp, i32, i32, i32, i32, vp, vp], C.c_int),
    "acn_hashgrid_bwd": ([vp, i64, vp, vp, i32, i32, i32, i32, vp, vp], C.c_int),
    "acn_sh_fwd": ([vp, i64, i32, vp, vp], C.c_int),
    "acn_workspace_bytes": ([i32], sz),
    "acn_pack_experts": ([vp, vp, i32, vp, sz, vp], C.c_int),
    "acn_field_fwd": ([vp, i64, i64, vp, vp, i32, vp, sz, vp, vp], C.c_int),
    "acn_volume_render_fwd": ([vp, vp, vp, i64, i32, i32, i32, f32, vp, vp, vp, vp, vp], C.c_int),
    "acn_render_stratified_fwd": ([vp, i64, i32, vp, vp, vp, i32, vp, f32, f32, vp, sz, vp, vp, vp, vp, vp],
                                  C.c_int),
    "acn_render_order_bytes": ([i64], sz),
    "acn_ray_order": ([vp, i64, vp, vp], C.c_int),
    "acn_routed_count_caps": ([vp, i64, i32, vp, vp, vp, vp, vp, vp, sz, vp], C.c_int),
    "acn_routed_count_caps_tiled": ([vp, i64, i32, vp, vp, vp, i32, vp, vp, vp, sz, vp], C.c_int),
    "acn_ep_gather_caps": ([vp, vp, i32, i32, vp, i32, vp, vp, f32, f32, vp, vp, vp, vp, vp, vp, vp, vp], C.c_int),
    "acn_ep_field_fwd": ([vp, vp, i32, i32, i64, vp, vp, sz, vp, vp], C.c_int),
    "acn_ep_field_fwd_compact": ([vp, vp, i32, i32, i64, i64, vp, vp, sz, vp, vp], C.c_int),
    "acn_routed_count_batches": ([vp, i64, i32, i64, vp, vp, vp, vp], C.c_int),
    "acn_ep_composite": ([vp, i64, i32, vp, vp, vp, vp, i32, i32, vp, f32, f32, vp, vp, vp, vp, vp], C.c_int),
    "acn_render_stratified_fwd_ordered": ([vp, i64, i32, vp, vp, vp, i32, vp, f32, f32, vp, sz, vp, vp, vp, vp,
                                           vp, sz, vp], C.c_int),
    "acn_get_rays": ([i32, i32, f32, f32, f32, f32, i32, vp, vp, f32, f32, i32, f32, i32, f32, i32, vp, vp, vp],
                     C.c_int),
    "acn_ray_directions": ([i32, i32, f32, f32, f32, f32, i32, vp, vp], C.c_int),
    "acn_rays_from_dirs": ([vp, i64, vp, vp, f32, f32, f32, f32, f32, vp, vp], C.c_int),
    "acn_ray_aabb": ([vp, vp, i64, vp, f32, f32, f32, vp, vp, vp], C.c_int),
    "acn_clamp_rays": ([vp, i64, i32, i32, f32, i32, f32, f32, f32, vp, vp], C.c_int),
    "acn_routing_fwd": ([vp, i64, i64, vp, vp, vp, vp], C.c_int),
    "acn_background_fwd": ([vp, i64, vp, vp, vp], C.c_int),
    "acn_background_bwd_workspace_bytes": ([], C.c_size_t),
    "acn_background_bwd": ([vp, i64, vp, vp, vp, vp, vp, vp, vp, C.c_size_t, vp], C.c_int),
    "acn_composite_mse_train_workspace_bytes": ([], C.c_size_t),
    "acn_routed_composite_mse_train": ([vp, i64, i32, vp, vp, vp, vp, i32, vp, i64, vp, vp, vp, vp, vp, vp, vp, vp,
                                        vp, vp, C.c_size_t, vp], C.c_int),
    "acn_volume_render_bwd": ([vp, vp, vp, i64, i32, f32, vp, vp, vp, vp, vp, vp, vp], C.c_int),
    "acn_grad_sumsq": ([vp, vp, i64, vp, vp, vp], C.c_int),
    "acn_mse_linear_fwd": ([vp, vp, i64, vp, vp], C.c_int),
    "acn_mse_linear_workspace_bytes": ([], C.c_size_t),
    "acn_mse_linear_fwd_ws": ([vp, vp, i64, vp, vp, C.c_size_t, vp], C.c_int),
    "acn_mse_linear_bwd": ([vp, vp, i64, vp, vp, vp], C.c_int),
    "acn_clip_coef": ([vp, f32, vp, vp], C.c_int),
    "acn_adam_step": ([vp, vp, i64, vp, i32, vp, vp], C.c_int),
    "acn_optim_plan_device": ([vp, i32, vp, vp, i64, vp], C.c_int),
    "acn_adam_table_bytes": ([i32, i32], C.c_size_t),
    "acn_adam_table_fill": ([vp, i32, i32, i32, vp, C.c_size_t], C.c_int),
    "acn_adam_step_table": ([vp, vp, i64, vp, i32, vp, i32, i32, vp, vp], C.c_int),
    "acn_occ_traverse": ([vp, i64, vp, i64, i64, vp, vp, vp, vp, i32, vp, f32, f32, vp, vp, i64, i64, vp, vp, vp, vp,
                          vp, vp],
                         C.c_int),
    "acn_occ_compact": ([vp, vp, i64, vp, vp, i64, vp, vp, vp, vp], C.c_int),
    "acn_occ_union": ([i32, i64, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp], C.c_int),
    "acn_render_packed_fwd": ([vp, i64, i64, vp, vp, vp, vp, vp, vp, i32, vp, vp, sz, vp, vp, vp, vp, vp], C.c_int),
    "acn_packed_weights_fwd": ([vp, vp, vp, vp, vp, i64, vp, vp, vp, vp], C.c_int),
    "acn_packed_weights_bwd": ([vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, i64, vp, vp], C.c_int),
    "acn_packed_accumulate_fwd": ([vp, vp, i32, vp, vp, i64, vp, vp], C.c_int),
    "acn_packed_accumulate_bwd": ([vp, vp, i32, vp, i64, vp, vp, vp, vp], C.c_int),
    "acn_occ_pack_bits": ([vp, i64, vp, vp], C.c_int),
    "acn_occ_cell_points": ([vp, i64, vp, vp, vp, vp, vp], C.c_int),
    "acn_occ_ema": ([vp, vp, vp, i64, f32, vp], C.c_int),
    "acn_occ_binarize_workspace_bytes": ([], sz),
    "acn_occ_binarize": ([vp, i64, f32, vp, vp, vp, vp, vp], C.c_int),
    "acn_occ_mark_invisible": ([vp, i32, vp, i32, i32, i32, f32, vp, vp, vp, i64, vp, vp], C.c_int),
    # data.hip
    "acn_route_rays": ([vp, i64, vp, vp, vp, vp, f32, f32, i32, i32, vp, vp, vp], C.c_int),
    "acn_bin_rays_workspace_bytes": ([i64, i32], C.c_size_t),
    "acn_bin_rays": ([vp, vp, i64, i32, vp, vp, vp, C.c_size_t, vp], C.c_int),
    # mlp_train.hip
    "acn_mlp_workspace_bytes": ([], C.c_size_t),
    "acn_mlp_train_fwd": ([vp, vp, i64, vp, vp, vp, vp, vp], C.c_int),
    "acn_mlp_train_bwd": ([vp, vp, vp, i64, vp, vp, vp, vp, vp], C.c_int),
    "acn_mlp_dw_workspace_bytes": ([], C.c_size_t),
    "acn_sample_stratified": ([vp, i64, C.c_int, vp, vp, vp, C.c_float, C.c_float, vp, vp, vp, vp], C.c_int),
    "acn_mlp_train_bwd_dw": ([vp, vp, vp, vp, i64, vp, vp, vp, vp, vp], C.c_int),
    "acn_mlp_train_bwd_dw_img": ([vp, vp, vp, vp, i64, vp, vp, vp, vp, vp], C.c_int),
    # routed.hip
    "acn_routed_workspace_bytes": ([i64, i32], C.c_size_t),
    "acn_routed_count": ([vp, i64, i32, vp, vp, i32, vp, vp, vp, sz, vp], C.c_int),
    "acn_routed_scatter": ([vp, i64, i32, i32, vp, vp, vp, vp, f32, f32, i32, vp, vp, vp, vp, vp, vp, vp, vp],
                           C.c_int),
    "acn_routed_blend_fwd": ([vp, vp, vp, i64, i32, vp, vp], C.c_int),
    "acn_routed_blend_bwd": ([vp, vp, vp, i64, vp, vp, vp], C.c_int),
    "acn_hashgrid_bwd_det_workspace_bytes": ([i64, i32, i32, i32], C.c_size_t),
    "acn_hashgrid_bwd_det": ([vp, i64, vp, vp, i32, i32, i32, i32, vp, vp, sz, vp], C.c_int),
    "acn_routed_scatter_xd": ([vp, i64, i32, i32, vp, vp, vp, vp, vp, vp, vp, vp, vp], C.c_int),
    "acn_routed_scatter_xd_tiled": ([vp, i64, i32, i32, i32, vp, vp, vp, vp, vp, vp, vp, vp, vp], C.c_int),
    "acn_routed_count_fixed": ([vp, i64, i32, vp, vp, i64, vp, vp, vp, sz, vp], C.c_int),
    "acn_routed_pad_pairs": ([vp, i32, i64, vp, vp, vp], C.c_int),
    "acn_ep_workspace_bytes": ([i32, i32], sz),
    "acn_ep_gather": ([vp, vp, i32, i32, i64, i32, vp, vp, f32, f32, vp, vp, vp, vp, vp, vp, vp, vp], C.c_int),
    "acn_ep_scatter_back": ([vp, vp, vp, i32, vp, vp], C.c_int),
    "acn_ep_gather_grad": ([vp, vp, vp, i32, vp, vp], C.c_int),
    "acn_xd_unit_sh": ([vp, i64, vp, vp, f32, f32, vp, vp, vp], C.c_int),
    "acn_hashgrid_fwd_pairs": ([vp, vp, vp, i32, vp, vp, i32, i32, i32, vp, vp], C.c_int),
    "acn_hashgrid_bwd_pairs": ([vp, vp, vp, vp, i32, vp, vp, vp, i32, i32, i32, vp], C.c_int),
    "acn_hashgrid_bwd_pairs_sumsq": ([vp, vp, vp, vp, i32, vp, vp, vp, i32, i32, i32, vp, vp], C.c_int),
    "acn_mlp_pairs_workspace_bytes": ([i32], C.c_size_t),
    "acn_mlp_pack_pairs": ([vp, i32, vp, vp], C.c_int),
    "acn_mlp_train_fwd_pairs": ([vp, vp, vp, i32, vp, vp, vp], C.c_int),
    "acn_mlp_train_bwd_dw_pairs": ([vp, vp, vp, vp, vp, i32, vp, vp, vp, vp], C.c_int),
    "acn_grad_sumsq_slots": ([vp, vp, i64, vp, vp, i32, vp, vp, vp], C.c_int),
    "acn_grad_sumsq_slots_ex": ([vp, vp, i64, vp, vp, i32, vp, vp, vp, vp], C.c_int),
    "acn_grad_clip_slots": ([vp, vp, i64, vp, vp, i32, vp, vp, vp, C.c_float, vp, vp, vp], C.c_int),
    "acn_adam_step_slots": ([vp, vp, i64, vp, vp, i32, i32, vp, i32, vp, i32, vp, vp], C.c_int),
    "acn_adam_step_slots_segmap": ([vp, vp, i64, vp, vp, i32, i32, vp, i32, vp, i32, vp, vp, vp], C.c_int),
    "acn_adam_step_slots_segmap_phase": ([vp, vp, i64, vp, vp, i32, i32, vp, i32, vp, i32, vp, vp, i32, vp], C.c_int),
    "acn_hashgrid_bwd_pairs_segmap": ([vp, vp, vp, vp, i32, vp, vp, vp, i32, i32, i32, vp, vp, vp], C.c_int),
    "acn_hashgrid_pairs_mark": ([vp, vp, vp, vp, i32, vp, i32, i32, i32, vp, vp], C.c_int),
    "acn_amp_unscale_coef": ([vp, f32, vp, vp, vp, f32, f32, i32, vp, vp, i32, vp], C.c_int),
    # clusters.hip
    "acn_voronoi_route": ([vp, i64, i32, vp, i32, i32, C.c_double, i32, i32, vp, vp, vp, vp, vp, vp], C.c_int),
}
# the exact-fp32 training MLP (suffix _exact) and the reference's use_amp arithmetic (suffix _amp): the same ten
# entry points (mlp_train.hip built three times)
MLP_ENTRY_POINTS = ("acn_mlp_workspace_bytes", "acn_mlp_train_fwd", "acn_mlp_train_bwd", "acn_mlp_dw_workspace_bytes",
                    "acn_mlp_train_bwd_dw", "acn_mlp_train_bwd_dw_img", "acn_mlp_pairs_workspace_bytes", "acn_mlp_pack_pairs",
                    "acn_mlp_train_fwd_pairs", "acn_mlp_train_bwd_dw_pairs")
SIGNATURES.update({n + sfx: SIGNATURES[n] for n in MLP_ENTRY_POINTS for sfx in ("_exact", "_amp")})


def lib():
    """Load libacnerf.so (once).  Raises if it is missing: there is no fallback path."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            if not LIB_PATH.exists():
                raise AcnError(f"libacnerf.so not found at {LIB_PATH}; build it with "
                               f"`python -c 'import __graft_entry__ as g; g.build()'` (or make -C "
                               f"adaptive_city_nerf_amd/csrc)")
            L = C.CDLL(str(LIB_PATH))
            variant = "ACNERF_LIB" in os.environ   # a developer build (tools/build_variants.sh) may predate an entry
            missing = []
            for name, (args, res) in SIGNATURES.items():
                if variant and not hasattr(L, name):
                    missing.append(name)
                    continue
                fn = getattr(L, name)
                fn.argtypes = args
                fn.restype = res
            if missing:
                _disable_fused_paths(missing)
            _lib = L
    return _lib


def _disable_fused_paths(missing) -> None:
    """A variant library without the fused entry points the defaults select: switch those paths off, loudly,
    instead of failing later with an AttributeError."""
    import warnings
    from . import optim, routed_train
    if "acn_grad_clip_slots" in missing and optim.FUSED_CLIP:
        optim.FUSED_CLIP = False
        warnings.warn(f"{LIB_PATH} lacks acn_grad_clip_slots: FUSED_CLIP switched off")
    if "acn_routed_composite_mse_train" in missing and routed_train.FUSED_COMPOSITE:
        routed_train.FUSED_COMPOSITE = False
        warnings.warn(f"{LIB_PATH} lacks acn_routed_composite_mse_train: FUSED_COMPOSITE switched off")


def exported_symbols():
    return list(SIGNATURES)


def check(status: int, what: str) -> None:
    if status != 0:
        buf = C.create_string_buffer(512)
        lib().acn_last_error(buf, 512)
        raise AcnError(f"{what} failed (status {status}): {buf.value.decode(errors='replace')}")


def ptr(t) -> int:
    return 0 if t is None else int(t.data_ptr())


def stream_of(t: torch.Tensor) -> int:
    return int(torch.cuda.current_stream(t.device).cuda_stream)


def require_hip(t: torch.Tensor, what: str) -> None:
    if not (isinstance(t, torch.Tensor) and t.is_cuda):
        raise AcnError(f"{what}: the HIP implementation needs tensors on a HIP device (got "
                       f"{getattr(t, 'device', type(t))}); there is no CPU fallback")


@contextlib.contextmanager
def graph_capture(graph, pool=None):
    """torch.cuda.graph(graph, pool) with Python's cyclic garbage collector held off: a collection inside the
    capture frees tensors of earlier, uncaptured work from within the capturing thread, which aborted the
    process on this stack (round 3, tests/test_meta_gpu.py region-without-tasks).  Garbage is collected just
    before the capture instead."""
    import gc
    gc.collect()
    was = gc.isenabled()
    gc.disable()
    keep = []
    _CAPTURE_KEEP.append(keep)
    try:
        with torch.cuda.graph(graph, pool=pool):
            yield
    finally:
        _CAPTURE_KEEP.pop()
        # buffers baked into this graph (per-capture workspaces: capture_keepalive) live as long as the graph
        graph._acn_keepalive = getattr(graph, "_acn_keepalive", []) + keep
        if was:
            gc.enable()


_CAPTURE_KEEP = []   # one list per active graph_capture


def capture_keepalive(t):
    """Tie ``t`` to the graph being captured (graph_capture): freed with the graph instead of living forever.
    Outside graph_capture (a bare torch.cuda.graph) it falls back to a module list."""
    if _CAPTURE_KEEP:
        _CAPTURE_KEEP[-1].append(t)
    else:
        _UNTRACKED_CAPTURE.append(t)
    return t


_UNTRACKED_CAPTURE = []
