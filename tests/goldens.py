"""Loading helpers for the committed golden fixtures (tests/golden/*.npz, allow_pickle=False)."""
from __future__ import annotations

import json
from functools import lru_cache
from pathlib import Path

import numpy as np

GOLDEN = Path(__file__).resolve().parent / "golden"
REPO = GOLDEN.parent.parent


@lru_cache(maxsize=None)
def load(name: str) -> dict:
    with np.load(GOLDEN / f"{name}.npz", allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


@lru_cache(maxsize=None)
def scene() -> dict:
    return json.loads((GOLDEN / "scene_drz_example.json").read_text())


MASK = {"k1": "g11_grid_bm110_ss11", "k4": "g22_grid_bm110_ss11"}


def expert_weights(d: dict, k: int, prefix: str = "w:") -> dict:
    pre = f"{prefix}submodules.{k}."
    return {key[len(pre):]: v for key, v in d.items() if key.startswith(pre)}


def fast_weights(d: dict, k: int) -> dict:
    return expert_weights(d, k, prefix="fast:")


def bg_weights(d: dict, prefix: str = "w:") -> dict:
    return {key[len(prefix):]: v for key, v in d.items() if key.startswith(prefix + "bg_mlp.")}


@lru_cache(maxsize=8)
def table(seed: int, scale: float, levels: int = 16, log2T: int = 20) -> np.ndarray:
    import sys
    sys.path.insert(0, str(REPO))
    from adaptive_city_nerf_amd.synthetic import formula_table
    return formula_table(levels, log2T, 2, seed=seed, scale=scale)
