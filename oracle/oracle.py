"""ctypes wrapper of the C oracle (acn_oracle.c) -- TEST INFRASTRUCTURE ONLY.

Imported only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg, always as the
checker, never as the thing measured or shipped.  The product package adaptive_city_nerf_amd never
imports this module.  Every function takes/returns numpy float32 arrays.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
from pathlib import Path
from typing import Dict, Optional, Sequence

import numpy as np

HERE = Path(__file__).resolve().parent
LIB_PATH = HERE / "build" / "liboracle.so"
_lib = None

f32p = np.ctypeslib.ndpointer(dtype=np.float32, flags="C_CONTIGUOUS")
i32p = np.ctypeslib.ndpointer(dtype=np.int32, flags="C_CONTIGUOUS")
u8p = np.ctypeslib.ndpointer(dtype=np.uint8, flags="C_CONTIGUOUS")


def build() -> Path:
    subprocess.run(["make", "-s", "-C", str(HERE)], check=True)
    return LIB_PATH


class OracleExpert(C.Structure):
    _fields_ = [
        ("table", C.c_void_p), ("res", C.c_void_p),
        ("L", C.c_int), ("log2T", C.c_int), ("F", C.c_int), ("interp", C.c_int),
        ("aabb_min", C.c_float * 3), ("aabb_extent", C.c_float * 3),
        ("n_sigma", C.c_int), ("hidden", C.c_int), ("geo_dim", C.c_int), ("n_color", C.c_int),
        ("color_hidden", C.c_int), ("sh_levels", C.c_int),
        ("sig_w", C.c_void_p * 8), ("sig_b", C.c_void_p * 8),
        ("sh_w", C.c_void_p), ("sh_b", C.c_void_p),
        ("geo_w", C.c_void_p), ("geo_b", C.c_void_p),
        ("col_w", C.c_void_p * 9), ("col_b", C.c_void_p * 9),
    ]


def lib():
    global _lib
    if _lib is None:
        if not LIB_PATH.exists():
            build()
        L = C.CDLL(str(LIB_PATH))
        L.oracle_hashgrid_fwd.argtypes = [f32p, C.c_int64, f32p, i32p, C.c_int, C.c_int, C.c_int, C.c_int, f32p]
        L.oracle_hashgrid_bwd.argtypes = [f32p, C.c_int64, f32p, i32p, C.c_int, C.c_int, C.c_int, C.c_int, f32p]
        L.oracle_sh_fwd.argtypes = [f32p, C.c_int64, C.c_int, f32p]
        L.oracle_expert_fwd.argtypes = [C.POINTER(OracleExpert), f32p, C.c_int64, C.c_int64, f32p]
        L.oracle_routing.argtypes = [f32p, C.c_int64, C.c_int64, f32p, C.c_int, C.c_int, C.c_float, C.c_void_p, C.c_void_p]
        L.oracle_container_fwd.argtypes = [C.POINTER(OracleExpert), C.c_int, f32p, C.c_int, C.c_float, C.c_int,
                                           f32p, C.c_int64, C.c_int64, f32p]
        L.oracle_volume_render.argtypes = [f32p, f32p, C.c_void_p, C.c_int64, C.c_int, C.c_int, C.c_int, C.c_float,
                                           f32p, f32p, C.c_void_p, f32p]
        L.oracle_render_stratified.argtypes = [f32p, C.c_int64, C.c_int, C.c_void_p, C.POINTER(OracleExpert), C.c_int,
                                               f32p, C.c_int, C.c_float, C.c_int, C.c_void_p, C.c_void_p, C.c_int,
                                               C.c_void_p, C.c_void_p, C.c_void_p, C.c_float, f32p, f32p, C.c_void_p, f32p]
        L.oracle_get_rays.argtypes = [C.c_int, C.c_int, C.c_float, C.c_float, C.c_float, C.c_float, C.c_int, f32p,
                                      C.c_void_p, C.c_float, C.c_float, C.c_int, C.c_float, C.c_int, C.c_float, C.c_int,
                                      f32p, u8p]
        L.oracle_max_threads.restype = C.c_int
        L.oracle_set_threads.argtypes = [C.c_int]
        _lib = L
    return _lib


def _c(a, dtype=np.float32):
    return np.ascontiguousarray(a, dtype=dtype)


def _ptr(a: Optional[np.ndarray]):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


def set_threads(n: int) -> None:
    lib().oracle_set_threads(int(n))


def max_threads() -> int:
    return int(lib().oracle_max_threads())


def level_resolutions(levels: int, min_res: int, max_res: int) -> np.ndarray:
    """encodings.py:202-215: floor(min_res * growth**arange(L) in float32) -> int32."""
    import math
    g = 1.0 if levels <= 1 else float(math.exp((math.log(max_res) - math.log(min_res)) / (levels - 1)))
    lv = np.arange(levels, dtype=np.float32)
    # torch computes growth_factor(python float) ** float32 tensor in float32 (pow), then floor
    import torch
    return torch.floor(min_res * (g ** torch.from_numpy(lv))).to(torch.int32).numpy()


def hashgrid_fwd(x01, table, res, L, log2T, F=2, interp=1):
    x01 = _c(x01).reshape(-1, 3); table = _c(table); res = _c(res, np.int32)
    out = np.empty((x01.shape[0], L * F), np.float32)
    lib().oracle_hashgrid_fwd(x01, x01.shape[0], table, res, L, log2T, F, interp, out)
    return out


def hashgrid_bwd(x01, gout, res, L, log2T, F=2, interp=1):
    x01 = _c(x01).reshape(-1, 3); gout = _c(gout); res = _c(res, np.int32)
    gt = np.empty((L << log2T, F), np.float32)
    lib().oracle_hashgrid_bwd(x01, x01.shape[0], gout, res, L, log2T, F, interp, gt)
    return gt


def sh_fwd(d, levels=4):
    d = _c(d).reshape(-1, 3)
    out = np.empty((d.shape[0], levels * levels), np.float32)
    lib().oracle_sh_fwd(d, d.shape[0], levels, out)
    return out


class Expert:
    """Holds numpy arrays alive and exposes the C struct.  `w` maps reference state-dict suffixes
    (e.g. 'sigma_trunk.0.linear.weight') to arrays."""

    def __init__(self, w: Dict[str, np.ndarray], table: np.ndarray, res: np.ndarray, aabb_min, aabb_extent,
                 log2T=20, F=2, interp=1, n_sigma=2, n_color=2, sh_levels=4):
        self.keep = []
        s = OracleExpert()
        tab = _c(table); r = _c(res, np.int32)
        self.keep += [tab, r]
        s.table = tab.ctypes.data; s.res = r.ctypes.data
        s.L = int(r.shape[0]); s.log2T = log2T; s.F = F; s.interp = interp
        s.aabb_min[:] = [float(v) for v in np.asarray(aabb_min, np.float32)]
        s.aabb_extent[:] = [float(v) for v in np.asarray(aabb_extent, np.float32)]

        def arr(k):
            a = _c(w[k]); self.keep.append(a); return a.ctypes.data

        s.n_sigma = n_sigma
        for i in range(n_sigma):
            s.sig_w[i] = arr(f"sigma_trunk.{i}.linear.weight"); s.sig_b[i] = arr(f"sigma_trunk.{i}.linear.bias")
        s.hidden = int(w["sigma_trunk.0.linear.weight"].shape[0]) if n_sigma else int(r.shape[0] * F)
        s.sh_w = arr("sigma_head.weight"); s.sh_b = arr("sigma_head.bias")
        s.geo_w = arr("geo_head.weight"); s.geo_b = arr("geo_head.bias")
        s.geo_dim = int(w["geo_head.weight"].shape[0])
        s.n_color = n_color
        for i in range(n_color):
            s.col_w[i] = arr(f"color_mlp.{i}.linear.weight"); s.col_b[i] = arr(f"color_mlp.{i}.linear.bias")
        s.col_w[n_color] = arr(f"color_mlp.{n_color}.weight"); s.col_b[n_color] = arr(f"color_mlp.{n_color}.bias")
        s.color_hidden = int(w["color_mlp.0.linear.weight"].shape[0]) if n_color else 0
        s.sh_levels = sh_levels
        self.s = s


def _expert_array(experts: Sequence[Expert]):
    arr = (OracleExpert * len(experts))(*[e.s for e in experts])
    return arr


def expert_fwd(expert: Expert, x_d):
    x_d = _c(x_d)
    out = np.empty((x_d.shape[0], 4), np.float32)
    lib().oracle_expert_fwd(C.byref(expert.s), x_d, x_d.shape[0], x_d.shape[1], out)
    return out


def routing(pts, centroids, cluster_2d=True, bm=1.05):
    pts = _c(pts); cent = _c(centroids)
    K = cent.shape[0]; M = pts.shape[0]
    W = np.empty((M, K), np.float32); hard = np.empty((M,), np.int32)
    lib().oracle_routing(pts, M, pts.shape[1], cent, K, int(cluster_2d), float(bm), _ptr(W), _ptr(hard))
    return (W, None) if bm > 1.0 else (None, hard.astype(np.int64))


def container_fwd(experts: Sequence[Expert], centroids, x_d, cluster_2d=True, bm=1.05, active_module=None):
    x_d = _c(x_d); cent = _c(centroids)
    arr = _expert_array(experts)
    out = np.empty((x_d.shape[0], 4), np.float32)
    lib().oracle_container_fwd(arr, len(experts), cent, int(cluster_2d), float(bm),
                               -1 if active_module is None else int(active_module), x_d, x_d.shape[0],
                               x_d.shape[1], out)
    return out


def volume_render(rgb_sigma, t_vals, bg=None, raw_rgb=False, raw_sigma=False, sigma_scale=1.0, want_weights=True):
    rs = _c(rgb_sigma); t = _c(t_vals)
    N, S = t.shape
    bgc = None if bg is None else _c(bg)
    rgb = np.empty((N, 3), np.float32); depth = np.empty((N,), np.float32); acc = np.empty((N,), np.float32)
    w = np.empty((N, S), np.float32) if want_weights else None
    lib().oracle_volume_render(rs, t, _ptr(bgc), N, S, int(raw_rgb), int(raw_sigma), float(sigma_scale),
                               rgb, depth, _ptr(w), acc)
    return rgb, depth, w, acc


def render_stratified(rays, S, experts: Sequence[Expert], centroids, cluster_2d=True, bm=1.05, active_module=None,
                      bg_mlp: Optional[Dict[str, np.ndarray]] = None, bg_const=None, jitter=None,
                      sigma_scale=1.0, want_weights=True):
    rays = _c(rays); cent = _c(centroids)
    N = rays.shape[0]
    arr = _expert_array(experts)
    keep = []
    bw1 = bb1 = bw2 = bb2 = None; H = 0
    if bg_mlp is not None:
        bw1 = _c(bg_mlp["bg_mlp.0.weight"]); bb1 = _c(bg_mlp["bg_mlp.0.bias"])
        bw2 = _c(bg_mlp["bg_mlp.2.weight"]); bb2 = _c(bg_mlp["bg_mlp.2.bias"]); H = bw1.shape[0]
    bgc = None if bg_const is None else _c(bg_const)
    jit = None if jitter is None else _c(jitter)
    keep += [bw1, bb1, bw2, bb2, bgc, jit]
    rgb = np.empty((N, 3), np.float32); depth = np.empty((N,), np.float32); acc = np.empty((N,), np.float32)
    w = np.empty((N, S), np.float32) if want_weights else None
    lib().oracle_render_stratified(rays, N, int(S), _ptr(jit), arr, len(experts), cent, int(cluster_2d), float(bm),
                                   -1 if active_module is None else int(active_module), _ptr(bw1), _ptr(bb1), H,
                                   _ptr(bw2), _ptr(bb2), _ptr(bgc), float(sigma_scale), rgb, depth, _ptr(w), acc)
    return rgb, depth, w, acc


def get_rays(H, W, fx, fy, cx, cy, c2w, aabb=None, center_pixels=True, near=None, far=None,
             near_far_override=None, apply_clamp=True):
    c2w = _c(np.asarray(c2w, np.float32)[:3, :4])
    ab = None if aabb is None else _c(aabb)
    rays = np.empty((H * W, 8), np.float32); valid = np.empty((H * W,), np.uint8)
    hn = hf = 0; nv = fv = 0.0
    if near_far_override is not None:
        if near_far_override[0] is not None: hn, nv = 1, float(near_far_override[0])
        if near_far_override[1] is not None: hf, fv = 1, float(near_far_override[1])
    lib().oracle_get_rays(int(H), int(W), float(fx), float(fy), float(cx), float(cy), int(center_pixels), c2w,
                          _ptr(ab), float(near or 0.0), float(far or 0.0), hn, nv, hf, fv, int(apply_clamp),
                          rays, valid)
    return rays, valid.astype(bool)
