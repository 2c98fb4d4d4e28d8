"""cluster_ref.py -- TEST INFRASTRUCTURE ONLY: CPU restatement of scripts/create_clusters.py.

Imported only by tests/ and bench.py's cpu_baseline leg, never by the product.

* per-ray routing and ray generation: cluster_oracle.c (see its header for the op order);
* centroids: _grid_centroids (:298-323), _kmeans_init / _run_kmeans (:326-377) -- torch CPU ops, the
  reference's own host arithmetic and generator calls;
* scene box and the final per-expert boxes of main (:650-700, :930-962).

Pinned by tests/golden/clusters.npz (made by running the reference's own functions and its main()
end to end on the CPU, tests/golden/make_golden.py gen_clusters).
"""
from __future__ import annotations

import ctypes as C
from typing import Optional, Tuple

import numpy as np
import torch

from . import oracle as O

F32 = np.float32
f32p = np.ctypeslib.ndpointer(dtype=np.float32, flags="C_CONTIGUOUS")
i64p = np.ctypeslib.ndpointer(dtype=np.int64, flags="C_CONTIGUOUS")
i32p = np.ctypeslib.ndpointer(dtype=np.int32, flags="C_CONTIGUOUS")
u8p = np.ctypeslib.ndpointer(dtype=np.uint8, flags="C_CONTIGUOUS")
u64p = np.ctypeslib.ndpointer(dtype=np.uint64, flags="C_CONTIGUOUS")
_bound = False


def _lib():
    global _bound
    L = O.lib()
    if not _bound:
        L.oracle_cluster_rays.argtypes = [C.c_int, C.c_int, C.c_float, C.c_float, C.c_float, C.c_float, C.c_int, f32p,
                                          f32p, C.c_int, C.c_float, C.c_int, C.c_float, f32p, u8p]
        L.oracle_voronoi.argtypes = [f32p, C.c_int64, C.c_int, f32p, C.c_int, C.c_int, C.c_int, C.c_double, C.c_int,
                                     u64p, f32p, f32p, i64p, i32p]
        _bound = True
    return L


def cluster_rays(H, W, fx, fy, cx, cy, center_pixels, c2w, aabb, near_far_override=(None, None)):
    rays = np.empty((H * W, 8), F32)
    valid = np.empty(H * W, np.uint8)
    n, f = near_far_override
    _lib().oracle_cluster_rays(int(H), int(W), float(fx), float(fy), float(cx), float(cy), int(center_pixels),
                               np.ascontiguousarray(np.asarray(c2w, F32)[:3, :4]), np.ascontiguousarray(aabb, F32),
                               int(n is not None), float(n or 0.0), int(f is not None), float(f or 0.0), rays, valid)
    return rays, valid.astype(bool)


def voronoi(rays, S, cents, cluster_2d, boundary_margin, orig=False, update=False, state=None):
    """-> bits (N,) uint64 and the (mins, maxs, counts, nan_flag) state (updated in place if given)."""
    rays = np.ascontiguousarray(rays, F32)
    cents = np.ascontiguousarray(cents, F32)
    Cn = cents.shape[0]
    if state is None:
        state = (np.full((Cn, 3), np.inf, F32), np.full((Cn, 3), -np.inf, F32), np.zeros(Cn, np.int64),
                 np.zeros(Cn, np.int32))
    mode = 2 if orig else (0 if boundary_margin == 1.0 else 1)
    bits = np.zeros(rays.shape[0], np.uint64)
    _lib().oracle_voronoi(rays, rays.shape[0], int(S), cents, Cn, int(bool(cluster_2d)), mode, float(boundary_margin),
                          int(bool(update) and not orig), bits, *state)
    return bits, state


def bits_to_mask(bits: np.ndarray, C: int) -> np.ndarray:
    return ((bits[:, None] >> np.arange(C, dtype=np.uint64)[None, :]) & np.uint64(1)).astype(bool)


# ------------------------------------------------------------------------------------- centroids
def grid_centroids(cam_pos: torch.Tensor, gx: int, gy: int, gz: int, cluster_2d: bool) -> torch.Tensor:
    if cam_pos.numel() == 0:
        return torch.zeros(((gy * gz) if cluster_2d else (gx * gy * gz), 3), dtype=torch.float32)
    lo, hi = cam_pos.min(0).values, cam_pos.max(0).values
    if cluster_2d:
        xm = (lo[0] + hi[0]) * 0.5
        Y = lo[1] + (torch.arange(gy) + 0.5) * ((hi[1] - lo[1]) / gy)
        Z = lo[2] + (torch.arange(gz) + 0.5) * ((hi[2] - lo[2]) / gz)
        YY, ZZ = torch.meshgrid(Y, Z, indexing="ij")
        return torch.stack((torch.full_like(YY, xm), YY, ZZ), -1).reshape(-1, 3)
    axes = [lo[a] + (torch.arange(g) + 0.5) * ((hi[a] - lo[a]) / max(g, 1)) for a, g in enumerate((gx, gy, gz))]
    return torch.stack(torch.meshgrid(*axes, indexing="ij"), -1).reshape(-1, 3)


def kmeans(points: torch.Tensor, K: int, iters: int, init: str, seed: int, weights: Optional[torch.Tensor]):
    g = torch.Generator(device="cpu").manual_seed(seed)
    if init == "random":
        cen = points[torch.randperm(points.size(0), generator=g)[:K]].clone()
    else:
        cen = torch.empty(K, points.size(1), dtype=points.dtype)
        if weights is None:
            cen[0] = points[torch.randint(points.size(0), (1,), generator=g)]
        else:
            cen[0] = points[torch.multinomial((weights / weights.sum()).cpu(), 1, generator=g)]
        for k in range(1, K):
            m2 = torch.cdist(points, cen[:k]).min(1).values ** 2
            p = (m2 * (weights if weights is not None else 1.0)).clamp_min_(1e-12)
            cen[k] = points[torch.multinomial(p / p.sum(), 1, generator=g)]
    w = weights if weights is not None else torch.ones(points.size(0), dtype=points.dtype)
    for _ in range(max(1, iters)):
        D = torch.cdist(points, cen)
        a = D.argmin(1)
        for k in range(K):
            m = a == k
            cen[k] = points[D[:, k].argmax()] if not m.any() else (w[m][:, None] * points[m]).sum(0) / w[m].sum()
    return cen


# ------------------------------------------------------------------------------------- boxes
def global_box(pose_scale: float, origin_x: float, alt_range, scene_scale: float, altitude_pad: float):
    lo_m, hi_m = sorted(map(float, alt_range))
    xa, xb = sorted((-hi_m, -lo_m))
    aabb = torch.tensor([[(xa - origin_x) / pose_scale, -scene_scale, -scene_scale],
                         [(xb - origin_x) / pose_scale, scene_scale, scene_scale]], dtype=torch.float32)
    p = torch.tensor([[altitude_pad / pose_scale, 0, 0]], dtype=torch.float32).view(-1, 3)[-1]
    return torch.stack([aabb[0] - p, aabb[1] + p], dim=0)


def final_boxes(mins, maxs, cnts, cents, aabb_g, box_margin: float = 0.0, pose_scale: float = 1.0,
                nan_flag=None) -> Tuple[torch.Tensor, torch.Tensor]:
    mins, maxs = torch.as_tensor(mins).clone(), torch.as_tensor(maxs).clone()
    if nan_flag is not None:
        nf = torch.as_tensor(nan_flag).bool()
        mins[nf] = float("nan")
        maxs[nf] = float("nan")
    lo, hi = aabb_g[0], aabb_g[1]
    mins, maxs = torch.maximum(mins, lo), torch.minimum(maxs, hi)
    empty = torch.as_tensor(cnts) == 0
    if empty.any():
        eps = torch.clamp((hi - lo).abs() * 1e-6, min=1e-7)
        cc = torch.minimum(torch.maximum(torch.as_tensor(cents, dtype=torch.float32), lo), hi)
        mins[empty] = torch.maximum(cc[empty] - eps, lo)
        maxs[empty] = torch.minimum(cc[empty] + eps, hi)
    if box_margin and box_margin > 0.0:
        m = float(box_margin) / pose_scale
        mins, maxs = torch.maximum(mins - m, lo), torch.minimum(maxs + m, hi)
    mins[:, 0] = lo[0]
    maxs[:, 0] = hi[0]
    return mins, maxs
