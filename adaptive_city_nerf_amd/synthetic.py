"""Deterministic synthetic parameters for parity fixtures and the benchmark.

The reference initialises its hash table with ``(torch.rand(T, F) * 2 - 1) * hash_init_scale``
(``models/encodings.py:264-268``).  A 128 MiB table cannot be committed as a fixture, so every
fixture and the benchmark fill the table from a closed-form counter hash instead: the value of
flat element ``i`` (row-major over ``(L*T, F)``) is

    u   = splitmix64(seed * 0x632BE59BD9B4E019 + i) >> 40          # 24-bit integer
    val = float32((u / 2**24 * 2 - 1) * scale)                      # computed in float64

so that any consumer (numpy here, the fixture generator, the GPU box) regenerates bit-identical
tables from ``(seed, scale)``.  This module is data plumbing, not part of the render path.
"""
from __future__ import annotations

import numpy as np

_GOLDEN = np.uint64(0x9E3779B97F4A7C15)
_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)
_SEED_MUL = np.uint64(0x632BE59BD9B4E019)


def splitmix64(z: np.ndarray) -> np.ndarray:
    """Vectorised splitmix64 finaliser on uint64 arrays (wrapping arithmetic)."""
    with np.errstate(over="ignore"):
        z = z + _GOLDEN
        z = (z ^ (z >> np.uint64(30))) * _M1
        z = (z ^ (z >> np.uint64(27))) * _M2
        return z ^ (z >> np.uint64(31))


def formula_uniform(n: int, seed: int, scale: float, start: int = 0) -> np.ndarray:
    """``n`` float32 values U(-scale, scale) for flat indices ``start .. start+n-1``."""
    out = np.empty(n, dtype=np.float32)
    block = 1 << 22
    with np.errstate(over="ignore"):
        base = np.uint64(seed) * _SEED_MUL
        for b0 in range(0, n, block):
            b1 = min(n, b0 + block)
            idx = np.arange(start + b0, start + b1, dtype=np.uint64) + base
            u = (splitmix64(idx) >> np.uint64(40)).astype(np.float64)
            out[b0:b1] = ((u / 16777216.0) * 2.0 - 1.0) * float(scale)
    return out


def formula_table(levels: int, log2_hashmap_size: int, features: int, seed: int,
                  scale: float) -> np.ndarray:
    """Hash table of shape ``(levels * 2**log2T, features)`` float32 (the reference layout)."""
    rows = levels * (1 << log2_hashmap_size)
    return formula_uniform(rows * features, seed, scale).reshape(rows, features)


def formula_table_rows(rows: np.ndarray, features: int, seed: int, scale: float) -> np.ndarray:
    """Values of selected table rows (for spot checks without materialising the table)."""
    rows = np.asarray(rows, dtype=np.uint64)
    flat = (rows[:, None] * np.uint64(features) + np.arange(features, dtype=np.uint64)[None, :])
    with np.errstate(over="ignore"):
        u = (splitmix64(flat + np.uint64(seed) * _SEED_MUL) >> np.uint64(40)).astype(np.float64)
    return (((u / 16777216.0) * 2.0 - 1.0) * float(scale)).astype(np.float32)


def grid_layout(gy: int, gz: int, example: dict, margin_frac: float = 0.0284) -> dict:
    """Synthetic ``g{gy}{gz}`` expert layout for configs the reference ships no mask set for
    (4x2).  Centroids follow ``_grid_centroids`` (scripts/create_clusters.py:298-323,
    cluster_2d): cell centres of a gy x gz grid over the camera-position box, x at its centre.
    The camera box is recovered from the shipped 2x2 layout (its centroids sit at 1/4 and 3/4 of
    the box).  Per-expert AABBs: the axis-aligned Voronoi cell of the grid, clipped to the global
    AABB and widened on interior faces by ``margin_frac`` of the global extent (the 2x2 example's
    boundary widening, scene_drz_example.json g22), x spanning the global box."""
    g22 = example["masks"]["g22_grid_bm110_ss11"]
    c = np.asarray(g22["centroids"], np.float64)
    lo_g, hi_g = np.asarray(g22["aabb_global"][0], np.float64), np.asarray(g22["aabb_global"][1], np.float64)
    ymin, ymax = c[:, 1].min(), c[:, 1].max()
    zmin, zmax = c[:, 2].min(), c[:, 2].max()
    ry, rz = 2.0 * (ymax - ymin), 2.0 * (zmax - zmin)          # centroids at 1/4, 3/4 of the range
    y0, z0 = ymin - ry / 4.0, zmin - rz / 4.0
    ys = y0 + (np.arange(gy) + 0.5) * ry / gy
    zs = z0 + (np.arange(gz) + 0.5) * rz / gz
    xc = float(c[0, 0])
    ybounds = np.concatenate([[lo_g[1]], 0.5 * (ys[1:] + ys[:-1]), [hi_g[1]]])
    zbounds = np.concatenate([[lo_g[2]], 0.5 * (zs[1:] + zs[:-1]), [hi_g[2]]])
    my, mz = margin_frac * (hi_g[1] - lo_g[1]), margin_frac * (hi_g[2] - lo_g[2])
    cents, mins, maxs = [], [], []
    for i in range(gy):
        for j in range(gz):
            cents.append([xc, ys[i], zs[j]])
            mins.append([lo_g[0], ybounds[i] - (my if i > 0 else 0.0), zbounds[j] - (mz if j > 0 else 0.0)])
            maxs.append([hi_g[0], ybounds[i + 1] + (my if i < gy - 1 else 0.0), zbounds[j + 1] + (mz if j < gz - 1 else 0.0)])
    f32 = lambda a: np.asarray(a, np.float32).tolist()  # noqa: E731
    return {"centroids": f32(cents), "cluster_2d": True, "boundary_margin": 1.1, "aabb_global": g22["aabb_global"],
            "mins": f32(mins), "maxs": f32(maxs)}
