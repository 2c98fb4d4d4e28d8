"""Tensor-level wrappers of the occupancy-grid entry points of libacnerf.so (include/acnerf.h,
csrc/occ.hip and the packed renderer in csrc/render.hip).

Packed sample lists are ray-major, as nerfacc 0.5.3 returns them: ray r owns the samples
[starts[r], starts[r] + counts[r]).  Two-pass producers (traversal, boundary union) count, scan on
device, then fill; the only host synchronisation is reading the total sample count to size the
outputs (nerfacc does the same).  No CPU path: CPU tensors raise.
"""
from __future__ import annotations

import ctypes as C
from typing import List, Optional, Sequence, Tuple

import torch

from . import _lib
from ._lib import AcnError, check, ptr, require_hip, stream_of
from .ops import _experts_array, _f32, pack_experts

I64 = torch.int64
# single-pass traversal: per-ray scratch rows of SINGLE_PASS_CAP samples while the scratch stays under
# SINGLE_PASS_SCRATCH_BYTES (larger batches, or a ray with more samples, take the count + fill passes)
SINGLE_PASS_CAP = 1024
SINGLE_PASS_SCRATCH_BYTES = 256 << 20


def _host_floats(vals) -> C.Array:
    v = [float(x) for x in vals]
    return (C.c_float * len(v))(*v)


def _host_res(res) -> C.Array:
    r = [int(x) for x in res]
    if len(r) != 3:
        raise AcnError(f"resolution must have 3 entries, got {r}")
    return (C.c_int32 * 3)(*r)


def scan_counts(counts: torch.Tensor) -> Tuple[torch.Tensor, int]:
    """Exclusive prefix sum of per-ray counts (device) and the total (one host read)."""
    if counts.numel() == 0:
        return counts.clone(), 0
    incl = torch.cumsum(counts, 0)
    return incl - counts, int(incl[-1].item())


def pack_bits(binaries: torch.Tensor) -> torch.Tensor:
    """One bit per cell of the bool occupancy buffer (flattened order), as int32 words."""
    require_hip(binaries, "OccGridEstimator")
    b = binaries.contiguous().view(-1)
    if b.dtype != torch.bool:
        b = b.to(torch.bool)
    n = b.numel()
    words = torch.empty((n + 31) // 32, device=b.device, dtype=torch.int32)
    check(_lib.lib().acn_occ_pack_bits(ptr(b), n, ptr(words), stream_of(b)), "acn_occ_pack_bits")
    return words


def traverse(rays_o: torch.Tensor, rays_d: torch.Tensor, near: torch.Tensor, far: torch.Tensor, bits: torch.Tensor,
             aabbs: Sequence[Sequence[float]], res: Sequence[int], step_size: float, cone_angle: float,
             prefilter: Optional[Sequence[float]] = None, prefilter_near_far: Optional[torch.Tensor] = None):
    """traverse_grids: (ray_indices (M,), t_starts (M,), t_ends (M,), starts (N,), counts (N,))."""
    require_hip(rays_o, "OccGridEstimator.sampling")
    assert rays_o.dim() == 2 and rays_o.shape[-1] >= 3, "rays_o must be (N,3)"
    assert rays_d.dim() == 2 and rays_d.shape[0] == rays_o.shape[0] and rays_d.shape[-1] >= 3, "rays_d must be (N,3)"
    dev = rays_o.device
    o = rays_o if (rays_o.dtype == torch.float32 and rays_o.stride(-1) == 1) else _f32(rays_o)
    d = rays_d if (rays_d.dtype == torch.float32 and rays_d.stride(-1) == 1) else _f32(rays_d)
    N = o.shape[0]
    nr, fr = _f32(near).view(-1), _f32(far).view(-1)
    L = len(aabbs)
    ab = _host_floats([v for a in aabbs for v in a])
    rs = _host_res(res)
    pf = None if prefilter is None else _host_floats(prefilter)
    pnf, ld_pf = None, 0
    if prefilter is not None:
        if prefilter_near_far is None or prefilter_near_far.stride(-1) != 1 or prefilter_near_far.dtype != torch.float32:
            raise AcnError("traverse: the prefilter needs an fp32 (N, 2) [near, far] view with unit column stride")
        pnf, ld_pf = prefilter_near_far, prefilter_near_far.stride(0)
    counts = torch.empty(N, device=dev, dtype=I64)
    lib = _lib.lib()
    s = stream_of(o)
    args = (ptr(o), o.stride(0), ptr(d), d.stride(0), N, ptr(nr), ptr(fr), ptr(bits), ab, L, rs, float(step_size),
            float(cone_angle), pf, ptr(pnf), ld_pf)
    cap = SINGLE_PASS_CAP if N * SINGLE_PASS_CAP * 8 <= SINGLE_PASS_SCRATCH_BYTES else 0
    if cap:  # single march into per-ray scratch rows, then a wave-per-ray compaction
        scratch = torch.empty(2, N, cap, device=dev, dtype=torch.float32)
        check(lib.acn_occ_traverse(*args, cap, ptr(counts), None, None, ptr(scratch[0]), ptr(scratch[1]), s),
              "acn_occ_traverse(single pass)")
        incl = torch.cumsum(counts, 0)
        M, cmax = [int(v) for v in torch.stack([incl[-1], counts.max()]).cpu()] if N else (0, 0)
        starts = incl - counts
    else:
        check(lib.acn_occ_traverse(*args, 0, ptr(counts), None, None, None, None, s), "acn_occ_traverse(count)")
        starts, M = scan_counts(counts)
        cmax = None
    ri = torch.empty(M, device=dev, dtype=I64)
    t0 = torch.empty(M, device=dev, dtype=torch.float32)
    t1 = torch.empty(M, device=dev, dtype=torch.float32)
    if M > 0:
        if cap and cmax <= cap:
            check(lib.acn_occ_compact(ptr(scratch[0]), ptr(scratch[1]), cap, ptr(counts), ptr(starts), N, ptr(ri),
                                      ptr(t0), ptr(t1), s), "acn_occ_compact")
        else:  # some ray overflowed its scratch row (or no scratch): march again straight into place
            check(lib.acn_occ_traverse(*args, 0, None, ptr(starts), ptr(ri), ptr(t0), ptr(t1), s),
                  "acn_occ_traverse(fill)")
    return ri, t0, t1, starts, counts


def union(lists: Sequence[Tuple[torch.Tensor, torch.Tensor, torch.Tensor, torch.Tensor]], N: int):
    """Boundary union of K packed lists [(starts_k (N,), counts_k (N,), t0_k, t1_k)] over the same N
    rays: (ray_indices, t_starts, t_ends, starts, counts)."""
    K = len(lists)
    if K < 1 or K > _lib.ACN_MAX_EXPERTS:
        raise AcnError(f"union of {K} lists is not supported (1..{_lib.ACN_MAX_EXPERTS})")
    dev = lists[0][0].device
    keep = [(_as_i64(s), _as_i64(c), _f32(a), _f32(b)) for s, c, a, b in lists]
    arr = lambda j: (C.c_void_p * K)(*[ptr(k[j]) for k in keep])  # noqa: E731
    st, ct, a0, a1 = arr(0), arr(1), arr(2), arr(3)
    counts = torch.empty(N, device=dev, dtype=I64)
    lib = _lib.lib()
    s = int(torch.cuda.current_stream(dev).cuda_stream)
    check(lib.acn_occ_union(K, N, st, ct, a0, a1, ptr(counts), None, None, None, None, s), "acn_occ_union(count)")
    starts, M = scan_counts(counts)
    ri = torch.empty(M, device=dev, dtype=I64)
    m0 = torch.empty(M, device=dev, dtype=torch.float32)
    m1 = torch.empty(M, device=dev, dtype=torch.float32)
    if M > 0:
        check(lib.acn_occ_union(K, N, st, ct, a0, a1, None, ptr(starts), ptr(ri), ptr(m0), ptr(m1), s),
              "acn_occ_union(fill)")
    return ri, m0, m1, starts, counts


def _as_i64(t: torch.Tensor) -> torch.Tensor:
    return t.detach().to(I64).contiguous()


# Optional timing hook (bench.py): pairs of events bracketing the fused packed render launch.
EVENT_HOOK = None


def render_packed(rays: torch.Tensor, starts: torch.Tensor, counts: torch.Tensor, t0: torch.Tensor, t1: torch.Tensor,
                  experts, routing, active_module: Optional[int], background, packed: Optional[torch.Tensor] = None,
                  want_weights: bool = True):
    """Fused occupancy render over packed samples: rgb (N,3), depth (N,), weights (M,) | None, acc (N,)."""
    require_hip(rays, "render_rays_occ")
    assert rays.dim() == 2 and rays.shape[-1] >= 6, "rays must be (N, >=6)"
    r = rays if (rays.dtype == torch.float32 and rays.stride(-1) == 1) else _f32(rays)
    N = r.shape[0]
    dev = r.device
    M = t0.numel()
    rgb = torch.empty(N, 3, device=dev, dtype=torch.float32)
    depth = torch.empty(N, device=dev, dtype=torch.float32)
    acc = torch.empty(N, device=dev, dtype=torch.float32)
    w = torch.empty(M, device=dev, dtype=torch.float32) if want_weights else None
    if N == 0:
        return rgb, depth, w, acc
    ws = packed if packed is not None else pack_experts(experts, routing, active_module)
    arr = _experts_array(experts)
    st, ct, a, b = _as_i64(starts), _as_i64(counts), _f32(t0), _f32(t1)
    hook = EVENT_HOOK
    if hook is not None:
        e0 = torch.cuda.Event(enable_timing=True)
        e0.record()
    check(_lib.lib().acn_render_packed_fwd(
        ptr(r), r.stride(0), N, ptr(st), ptr(ct), ptr(a), ptr(b), arr, C.byref(routing),
        -1 if active_module is None else int(active_module), C.byref(background), ptr(ws), ws.numel() * 4,
        ptr(rgb), ptr(depth), ptr(w), ptr(acc), stream_of(r)), "acn_render_packed_fwd")
    if hook is not None:
        e1 = torch.cuda.Event(enable_timing=True)
        e1.record()
        hook.append((e0, e1))
    return rgb, depth, w, acc


def packed_weights(sigmas, t0, t1, starts, counts):
    sg, a, b = _f32(sigmas).view(-1), _f32(t0).view(-1), _f32(t1).view(-1)
    st, ct = _as_i64(starts), _as_i64(counts)
    M = sg.numel()
    w = torch.empty(M, device=sg.device, dtype=torch.float32)
    tr = torch.empty_like(w)
    al = torch.empty_like(w)
    check(_lib.lib().acn_packed_weights_fwd(ptr(sg), ptr(a), ptr(b), ptr(st), ptr(ct), st.numel(), ptr(w), ptr(tr),
                                            ptr(al), stream_of(sg)), "acn_packed_weights_fwd")
    return w, tr, al


def packed_weights_bwd(sigmas, t0, t1, w, tr, al, g_w, g_tr, g_al, starts, counts):
    sg = _f32(sigmas).view(-1)
    st, ct = _as_i64(starts), _as_i64(counts)
    gs = torch.empty_like(sg)
    f = lambda t: None if t is None else _f32(t).view(-1)  # noqa: E731
    check(_lib.lib().acn_packed_weights_bwd(ptr(sg), ptr(f(t0)), ptr(f(t1)), ptr(f(w)), ptr(f(tr)), ptr(f(al)),
                                            ptr(f(g_w)), ptr(f(g_tr)), ptr(f(g_al)), ptr(st), ptr(ct), st.numel(),
                                            ptr(gs), stream_of(sg)), "acn_packed_weights_bwd")
    return gs


def packed_accumulate(w, values, starts, counts):
    ww = _f32(w).view(-1)
    st, ct = _as_i64(starts), _as_i64(counts)
    N = st.numel()
    v = None if values is None else _f32(values).view(ww.numel(), -1)
    Cc = 1 if v is None else v.shape[1]
    out = torch.empty(N, Cc, device=ww.device, dtype=torch.float32)
    check(_lib.lib().acn_packed_accumulate_fwd(ptr(ww), ptr(v), Cc, ptr(st), ptr(ct), N, ptr(out), stream_of(ww)),
          "acn_packed_accumulate_fwd")
    return out


def packed_accumulate_bwd(w, values, ray_indices, g_out, need_w: bool, need_v: bool):
    ww = _f32(w).view(-1)
    M = ww.numel()
    v = None if values is None else _f32(values).view(M, -1)
    Cc = 1 if v is None else v.shape[1]
    g = _f32(g_out).view(-1, Cc)
    gw = torch.empty(M, device=ww.device, dtype=torch.float32) if need_w else None
    gv = torch.empty(M, Cc, device=ww.device, dtype=torch.float32) if (need_v and v is not None) else None
    check(_lib.lib().acn_packed_accumulate_bwd(ptr(ww), ptr(v), Cc, ptr(_as_i64(ray_indices)), M, ptr(g), ptr(gw),
                                               ptr(gv), stream_of(ww)), "acn_packed_accumulate_bwd")
    return gw, gv


def cell_points(cell_indices: torch.Tensor, u: Optional[torch.Tensor], aabb: Sequence[float], res) -> torch.Tensor:
    idx = _as_i64(cell_indices)
    n = idx.numel()
    x = torch.empty(n, 3, device=idx.device, dtype=torch.float32)
    uu = None if u is None else _f32(u).view(n, 3)
    check(_lib.lib().acn_occ_cell_points(ptr(idx), n, ptr(uu), _host_floats(aabb), _host_res(res), ptr(x),
                                         stream_of(idx)), "acn_occ_cell_points")
    return x


def ema(occs: torch.Tensor, cell_ids: torch.Tensor, occ: torch.Tensor, decay: float) -> None:
    if occs.dtype != torch.float32 or not occs.is_contiguous():
        raise AcnError("occs must be a contiguous float32 buffer")
    ids, o = _as_i64(cell_ids), _f32(occ).view(-1)
    if o.numel() != ids.numel():
        raise AcnError(f"occ_eval_fn returned {o.numel()} values for {ids.numel()} cells")
    check(_lib.lib().acn_occ_ema(ptr(occs), ptr(ids), ptr(o), ids.numel(), float(decay), stream_of(occs)),
          "acn_occ_ema")


def binarize(occs: torch.Tensor, occ_thre: float, binaries: torch.Tensor, bits: Optional[torch.Tensor]) -> torch.Tensor:
    """binaries <- occs > min(mean(occs[occs >= 0]), occ_thre), in place; returns the threshold (device)."""
    if not (binaries.dtype == torch.bool and binaries.is_contiguous() and binaries.numel() == occs.numel()):
        raise AcnError("binaries must be a contiguous bool buffer with one entry per cell")
    nb = int(_lib.lib().acn_occ_binarize_workspace_bytes())
    ws = torch.empty(nb // 8, device=occs.device, dtype=torch.float64)
    thre = torch.empty(1, device=occs.device, dtype=torch.float32)
    check(_lib.lib().acn_occ_binarize(ptr(occs), occs.numel(), float(occ_thre), ptr(binaries), ptr(bits), ptr(thre),
                                      ptr(ws), stream_of(occs)), "acn_occ_binarize")
    return thre


def mark_invisible(Ks: torch.Tensor, c2w: torch.Tensor, width: int, height: int, near_plane: float,
                   aabb: Sequence[float], res, cell_indices: torch.Tensor, occs_level: torch.Tensor) -> None:
    k = _f32(Ks).view(-1, 3, 3)
    p = _f32(c2w)[:, :3, :4].contiguous()
    idx = _as_i64(cell_indices)
    check(_lib.lib().acn_occ_mark_invisible(ptr(k), k.shape[0], ptr(p), p.shape[0], int(width), int(height),
                                            float(near_plane), _host_floats(aabb), _host_res(res), ptr(idx),
                                            idx.numel(), ptr(occs_level), stream_of(k)), "acn_occ_mark_invisible")
