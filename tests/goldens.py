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


MASK = {"k1": "g11_grid_bm110_ss11", "k4": "g22_grid_bm110_ss11", "k8": "g42_synthetic"}


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


# ------------------------------------------------------------------ data_tasks.npz (gen_data)
# name: (region, cells, alpha, policy, seed, TaskDataset kwargs) -- make_golden.py TASK_CASES
TASK_CASES = {
    "runner": (0, dict(S_target=512, Q_target=256, min_rays_cell=384, image_cap=0.4, assignment_checkpoint=0.7,
                       routing_policy="dda", cells=(1, 5, 5), seed=0)),
    "alpha_box": (0, dict(S_target=400, Q_target=200, min_rays_cell=600, image_cap=None, routing_policy="alpha",
                          max_images_support=2, max_images_query=1, cells=(1, 6, 6), seed=3, region_box=True)),
    "small_alpha": (2, dict(S_target=300, Q_target=150, min_rays_cell=200, image_cap=0.4, routing_policy="alpha",
                            cells=(2, 3, 3), seed=7, max_images_query=1, min_images_support=3)),
}


def data_masks(d: dict, region: int):
    shp = tuple(int(v) for v in d[f"r{region}_mask_shape"])
    return [np.unpackbits(m)[: shp[0] * shp[1]].reshape(shp).astype(bool) for m in d[f"r{region}_masks"]]


def task_kwargs(d: dict, name: str):
    """(region, TaskDataset kwargs with region_bounds resolved)."""
    region, kw = TASK_CASES[name]
    kw = dict(kw)
    if kw.pop("region_box", False):
        kw["region_bounds"] = tuple(tuple(float(v) for v in row) for row in d["box_aabbs"][region])
    return region, kw


def split_pools(d: dict, name: str):
    counts = d[f"t_{name}_counts"]
    flat = d[f"t_{name}_flat_idx"]
    return np.split(flat, np.cumsum(counts)[:-1])


def episodes(d: dict, name: str):
    """[(block_id, support idx, query idx, image_disjoint_ok, n_warnings)] of the reference run."""
    ep = d[f"t_{name}_episodes"]
    s = np.split(d[f"t_{name}_support"], np.cumsum(ep[:, 1])[:-1])
    q = np.split(d[f"t_{name}_query"], np.cumsum(ep[:, 2])[:-1])
    return [(int(e[0]), s[i], q[i], int(e[3]), int(e[4])) for i, e in enumerate(ep)]


def write_data_scene(root: Path, d: dict, region: int, scale: float = 0.125) -> Path:
    """The fixture as a COLMAP-converted layout (train/metadata/*.pt, train/rgbs/*.png at the target
    size so no resize happens, masks/<set>/<region>/<stem>.pt zipped like the reference's), with
    filler metadata so the image indices equal the reference's.  Returns the region's mask dir."""
    import zipfile

    import torch
    from PIL import Image

    stems = [str(s) for s in d["stems"]]
    (root / "train" / "metadata").mkdir(parents=True, exist_ok=True)
    (root / "train" / "rgbs").mkdir(parents=True, exist_ok=True)
    mdir = root / "masks" / "fixture" / str(region)
    mdir.mkdir(parents=True, exist_ok=True)
    H, W = [int(v) for v in d["HW"]]
    for j in range(int(d["image_index"].max()) + 1):
        name = f"{j:06d}"
        if name not in stems:  # metadata without an image: skipped by get_metadata_item
            torch.save({"c2w": torch.eye(3, 4), "W": 1, "H": 1, "intrinsics": torch.ones(4)},
                       root / "train" / "metadata" / f"{name}.pt")
    for i, stem in enumerate(stems):
        torch.save({"c2w": torch.from_numpy(d["c2w"][i]), "W": round(W / scale), "H": round(H / scale),
                    "intrinsics": torch.from_numpy(d["intrinsics"][i]) / scale},
                   root / "train" / "metadata" / f"{stem}.pt")
        Image.fromarray(d["images"][i]).save(root / "train" / "rgbs" / f"{stem}.png")
    for stem, m in zip(stems, data_masks(d, region)):
        inner = root / f"{stem}.inner.pt"
        torch.save(torch.from_numpy(m), inner)
        with zipfile.ZipFile(mdir / f"{stem}.pt", "w") as zf:
            zf.write(inner, arcname=f"{stem}.pt")
        inner.unlink()
    return mdir
