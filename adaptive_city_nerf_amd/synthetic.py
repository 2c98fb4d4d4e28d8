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
