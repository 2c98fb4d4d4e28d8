"""Device-resident ray tables and episodic task sampling.

Mirrors the reference's data layer around the hot path:

* ``ImageMetadata`` / ``get_image_metadata`` (data/image_metadata.py:41-123, data/dataset.py:185-291):
  camera + image + per-region mask records of a COLMAP-converted scene (``{split}/metadata/*.pt``,
  ``{split}/rgbs/*.jpg``, ``masks/<set>/<region>/<stem>.pt`` possibly zipped).  Serialized files are
  read with ``torch.load(weights_only=True)``.
* ``DeviceRaysDataset`` -- the RamRaysDataset (data/ram_rays_dataset.py:127-258) with the per-image
  work on the GPU: the JPEG is decoded on the host (PIL, as the reference), uploaded as uint8, and
  ONE fused HIP launch (acn_get_rays: get_ray_directions + get_rays + SceneBox slab test +
  clamp_rays_near_far) produces every pixel's ray; mask + validity compaction and the /255 happen on
  the device, and the concatenated table (``_rays`` (N,8), ``_rgbs`` (N,3), ``_img_indices`` (N,))
  lives in HBM -- no process pool, no host copy of the rays.
* ``TaskDataset`` -- data/task_dataset.py:29-1004: rays of one region are routed to micro-cells by
  the HIP kernel ``acn_route_rays`` (alpha-point + 6-neighbour max overlap, or the 64-step DDA max
  overlap, and the selected-cell overlap tolerance: bit-for-bit the reference's assignments), binned
  by a stable device sort, and episodes (support / query splits with the image-disjointness and
  per-image cap rules) are drawn with the reference's host generator in the reference's call order,
  then gathered from the device table.
"""
from __future__ import annotations

import ctypes as C
import math
import warnings
from dataclasses import dataclass, field
from pathlib import Path
from typing import Dict, List, Optional, Sequence, Tuple
from zipfile import ZipFile

import torch
import torch.nn.functional as F
from torch.utils.data import Dataset, IterableDataset

from . import _lib, ops
from ._lib import AcnError, check, ptr, stream_of

_RADIX_SORT_MIN = 32768  # torch CPU sort: stable radix path from at::internal::GRAIN_SIZE elements
_U8_TABLES: Dict[torch.device, torch.Tensor] = {}


def _u8_unit_table(device) -> torch.Tensor:
    t = _U8_TABLES.get(device)
    if t is None:
        t = _U8_TABLES[device] = torch.arange(256, dtype=torch.uint8).to(torch.float32).div_(255.0).to(device)
    return t



# =============================================================================== metadata
class ImageMetadata:
    """One posed image (data/image_metadata.py:41-123): c2w (3,4) RUB, intrinsics [fx, fy, cx, cy]."""

    def __init__(self, image_path: Path, c2w: torch.Tensor, W: int, H: int, intrinsics: torch.Tensor,
                 image_index: int, is_val=False, mask_dir: Optional[Path] = None):
        self.image_path = image_path
        self.c2w = c2w
        self.W = W
        self.H = H
        self.intrinsics = intrinsics
        self.image_index = image_index
        self.is_val = is_val
        self.mask_path = (Path(mask_dir) / f"{Path(image_path).stem}.pt") if mask_dir is not None else None

    def load_image(self) -> torch.Tensor:
        """(H, W, 3) uint8 RGB, LANCZOS-resized to (W, H) when the file differs."""
        from PIL import Image
        import numpy as np
        img = Image.open(self.image_path).convert("RGB")
        if img.size != (self.W, self.H):
            img = img.resize((self.W, self.H), Image.LANCZOS)
        return torch.from_numpy(np.array(img, dtype=np.uint8))

    def load_mask(self) -> Optional[torch.Tensor]:
        """(H, W) bool keep-mask, nearest-resized; None if the file is missing or malformed."""
        if self.mask_path is None or not self.mask_path.exists():
            return None
        try:
            m = torch.load(self.mask_path, map_location="cpu", weights_only=True)
        except Exception:
            with ZipFile(self.mask_path, "r") as zf, zf.open(zf.namelist()[0]) as f:
                m = torch.load(f, map_location="cpu", weights_only=True)
        if m.ndim == 1:
            if m.numel() != self.H * self.W:
                return None
            m = m.view(self.H, self.W)
        if m.ndim != 2:
            return None
        if tuple(m.shape) != (self.H, self.W):
            m = F.interpolate(m[None, None].float(), size=(self.H, self.W), mode="nearest")[0, 0]
        return m.bool()


def _metadata_files(d: Path) -> List[Path]:
    return sorted(d.glob("*.pt")) if d.exists() else []


def get_metadata_item(metadata_path: Path, image_index: int, scale_factor: float, is_val: bool = False,
                      mask_dir: Optional[Path] = None) -> Optional[ImageMetadata]:
    """data/dataset.py:257-291: the record of one metadata/*.pt and its rgbs/ image."""
    image_path = next((p for ext in (".jpg", ".JPG", ".png", ".PNG")
                       for p in [metadata_path.parent.parent / "rgbs" / f"{metadata_path.stem}{ext}"] if p.exists()),
                      None)
    if image_path is None:
        return None
    md = torch.load(metadata_path, map_location="cpu", weights_only=True)
    return ImageMetadata(image_path, md["c2w"], int(round(md["W"] * scale_factor)), int(round(md["H"] * scale_factor)),
                         md["intrinsics"] * scale_factor, image_index, is_val, mask_dir)


def get_image_metadata(data_path: str, scale_factor: float, mask_dir: Optional[str] = None,
                       only_test: bool = False) -> Tuple[List[ImageMetadata], List[ImageMetadata]]:
    """data/dataset.py:185-254: (train_items, val_items) of a flat or split COLMAP-converted layout;
    image indices enumerate all metadata files sorted by name."""
    root = Path(data_path)
    flat = _metadata_files(root / "metadata")
    if flat and (root / "rgbs").exists():
        index = {p.name: i for i, p in enumerate(sorted(flat, key=lambda x: x.name))}
        return [], [get_metadata_item(p, index[p.name], scale_factor, True, mask_dir) for p in flat]
    train = _metadata_files(root / "train" / "metadata")
    evals = _metadata_files(root / "val" / "metadata") or _metadata_files(root / "test" / "metadata")
    if not (train or evals):
        return [], []
    index = {p.name: i for i, p in enumerate(sorted(train + evals, key=lambda x: x.name))}
    tr = [] if only_test else [get_metadata_item(p, index[p.name], scale_factor, False, mask_dir) for p in train]
    return tr, [get_metadata_item(p, index[p.name], scale_factor, True, mask_dir) for p in evals]


# =============================================================================== ray table
def meganerf_val_balancing(keep_mask: torch.Tensor, H: int, W: int) -> torch.Tensor:
    """Mega-NeRF validation balancing (ram_rays_dataset.py:232-258): the right half is held out and
    as many random pixels of the left half are added (global generator, as the reference)."""
    keep = keep_mask.view(H, W).clone()
    left = keep[:, : W // 2]
    n_right = int(keep[:, W // 2:].sum().item())
    if n_right > 0:
        cand = torch.arange(H * W, device=keep.device).view(H, W)[:, : W // 2][~left]
        if cand.numel() > 0:
            add = cand[torch.randperm(cand.numel(), device=keep.device)[:n_right]]
            keep.view(-1).scatter_(0, add, torch.ones_like(add, dtype=torch.bool))
    keep[:, W // 2:] = False
    return keep.view(-1).bool()


class DeviceRaysDataset(Dataset):
    """RamRaysDataset on the GPU: ``_rays`` (N,8), ``_rgbs`` (N,3) fp32 in [0,1], ``_img_indices``
    (N,) int32 -- every kept, valid pixel of every image, in image order then row-major."""

    def __init__(self, metadata_items: Sequence, center_pixels: bool, val_balancing: bool = False,
                 ray_gen_kwargs: Optional[dict] = None, num_workers: Optional[int] = None, device=None):
        super().__init__()
        if ray_gen_kwargs is None or "scene_box" not in ray_gen_kwargs:
            raise ValueError("ray_gen_kwargs must contain keys: 'scene_box' and 'near_far_override'")
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        box = ray_gen_kwargs["scene_box"]
        override = ray_gen_kwargs.get("near_far_override", None)
        rgbs, rays, idx = [], [], []
        with torch.no_grad():
            for md in metadata_items:
                out = self._process(md, center_pixels, val_balancing, box, override)
                if out is not None:
                    rgbs.append(out[0]); rays.append(out[1]); idx.append(out[2])
        if not rgbs:
            warnings.warn("DeviceRaysDataset ended up empty. Check masks/val logic.")
            self._rgbs = torch.zeros((0, 3), dtype=torch.float32, device=self.device)
            self._rays = torch.zeros((0, 8), dtype=torch.float32, device=self.device)
            self._img_indices = torch.zeros((0,), dtype=torch.int32, device=self.device)
            self._num_images = 0
            return
        self._rgbs = torch.cat(rgbs, 0).contiguous()
        self._rays = torch.cat(rays, 0).contiguous()
        self._img_indices = torch.cat(idx, 0).contiguous()
        self._num_images = len(rgbs)
        self._img_unique_ids = torch.unique(self._img_indices).cpu().tolist()

    def _process(self, md, center_pixels, val_balancing, box, override):
        """One image (ram_rays_dataset.py:46-121): fused HIP ray generation + device compaction."""
        if md is None:
            return None
        img = md.load_image()
        if img is None:
            return None
        if img.ndim == 3 and img.shape[0] == 3 and img.shape[-1] != 3:
            img = img.permute(1, 2, 0).contiguous()
        if not (img.ndim == 3 and img.shape[-1] == 3) and not (img.ndim == 2 and img.shape[-1] == 3):
            return None
        keep = md.load_mask()
        if keep is not None and keep.ndim == 1:
            keep = keep.view(md.H, md.W)
        if getattr(md, "is_val", False) and val_balancing:
            if keep is None:
                keep = torch.ones(md.H, md.W, dtype=torch.bool)
            keep = meganerf_val_balancing(keep, md.H, md.W)
        if keep is not None and int(keep.sum().item()) == 0:
            return None
        fx, fy, cx, cy = [float(v) for v in md.intrinsics]
        rays, valid = ops.get_rays_image(md.H, md.W, fx, fy, cx, cy, md.c2w, box.aabb, self.device,
                                         center_pixels=center_pixels, near_far_override=override,
                                         apply_clamp=override is not None)
        sel = valid if keep is None else (valid & keep.reshape(-1).to(self.device, non_blocking=True))
        rays = rays[sel]
        if rays.shape[0] == 0:
            return None
        # u8 -> [0, 1] through a 256-entry table made with the reference's own host op (x.float() / 255):
        # the device's scalar division multiplies by the reciprocal, 1 ulp off for ~45% of values
        lut = _u8_unit_table(self.device)
        rgb = lut[img.reshape(-1, 3).to(self.device, non_blocking=True)[sel].long()]
        return rgb, rays, torch.full((rays.shape[0],), int(md.image_index), dtype=torch.int32, device=self.device)

    def __len__(self) -> int:
        return self._rgbs.shape[0]

    def __getitem__(self, idx) -> Dict[str, torch.Tensor]:
        return {"rgbs": self._rgbs[idx], "rays": self._rays[idx], "img_indices": self._img_indices[idx]}


def discover_cluster_cells(mask_dir: Path) -> int:
    """Region count of a mask set: params.pt centroids, else numbered sub-folders (utils.py:649-658)."""
    mask_dir = Path(mask_dir)
    subdirs = len([p for p in mask_dir.iterdir() if p.is_dir()])
    params = mask_dir / "params.pt"
    if params.exists():
        return len(torch.load(params, map_location="cpu", weights_only=True).get("centroids", [])) or subdirs
    return subdirs


def cap_metadata(md_list, cap_images):
    """Random subset of ``cap_images`` records (global generator) (data/dataset.py:147-154)."""
    if cap_images is None or cap_images <= 0 or len(md_list) <= cap_images:
        return md_list
    return [md_list[i] for i in torch.randperm(len(md_list))[:cap_images].tolist()]


def get_meta_lookups(train_md, val_md):
    """{image_index: {"H", "W"}} per split (data/dataset.py:157-172)."""
    look = lambda mds: {md.image_index: {"H": md.H, "W": md.W} for md in mds} if mds else None  # noqa: E731
    return look(train_md), look(val_md)


def get_dataset(P, dataset: str, only_test: bool = False, ray_gen_kwargs: Optional[dict] = None, device=None):
    """data/dataset.py:8-141 on the device: the full-scene (train, val) pair, or -- with
    ``P.mask_dirname`` -- per-region (train_sets, val_sets) lists of DeviceRaysDataset, region k's
    rays bounded by ``ray_gen_kwargs["expert_box_list"][k]`` and filtered by its masks."""
    if dataset != "drz":
        raise NotImplementedError()
    P.data_size = None
    data_path = Path(P.data_path) / "out" / P.data_dirname
    kw = dict(ray_gen_kwargs or {})
    if getattr(P, "mask_dirname", None) is None:
        train_md, val_md = get_image_metadata(data_path, P.downscale, mask_dir=None)
        args = {"center_pixels": True, "ray_gen_kwargs": kw, "device": device}
        train_set = DeviceRaysDataset(train_md, **args)
        test_set = DeviceRaysDataset(val_md, **args)
        return test_set if only_test else (train_set, test_set)
    mask_root = data_path / "masks" / P.mask_dirname
    n_cells = discover_cluster_cells(mask_root)
    assert n_cells == P.num_submodules, (f"Mismatch. Mask directory contains {n_cells} regions but the experiment is "
                                         f"configured for {P.num_submodules}.")
    boxes = kw.pop("expert_box_list")
    train_sets, val_sets = [], []
    for cell_id in range(P.num_submodules):
        train_md, val_md = get_image_metadata(data_path, P.downscale, mask_root / f"{cell_id}", only_test)
        if not train_md and not val_md:
            continue
        if getattr(P, "cap_images", None) is not None:
            train_md, val_md = cap_metadata(train_md, P.cap_images), cap_metadata(val_md, P.cap_images)
        args = {"center_pixels": True, "ray_gen_kwargs": dict(kw, scene_box=boxes[cell_id]), "device": device}
        tr = None if only_test else DeviceRaysDataset(train_md, **args)
        va = DeviceRaysDataset(val_md, **args) if val_md else None
        if tr is not None and len(tr) > 0:
            train_sets.append(tr)
        if va is not None and len(va) > 0:
            val_sets.append(va)
    P.dim_in, P.dim_out = 6, 4
    P.data_type = "ray"
    return train_sets, val_sets


# =============================================================================== episodes
@dataclass
class Task:
    """One episode: support/query sampled from a single spatial cell (task_dataset.py:11-22)."""
    support: Dict[str, torch.Tensor]
    query: Dict[str, torch.Tensor]
    cell_id: Optional[int] = None
    block_id: Optional[int] = None
    bounds: Optional[torch.Tensor] = None
    support_imgs: Optional[List[int]] = None
    query_imgs: Optional[List[int]] = None
    warnings: List[str] = field(default_factory=list)
    metrics: Dict[str, float] = field(default_factory=dict)


def cell_grid(aabb: torch.Tensor, cells: Tuple[int, int, int]) -> Tuple[torch.Tensor, torch.Tensor]:
    """Micro-cell AABBs (C,2,3) and sizes (C,3) of a region, x-major then y then z
    (task_dataset.py:174-195), evaluated on the host like the reference (its rays live on the CPU)."""
    aabb = aabb.detach().float().cpu()
    lo, hi = aabb[0], aabb[1]
    size = (hi - lo).clamp(min=1e-9)
    axes = [torch.linspace(0, 1, steps=n + 1) for n in cells]
    lo_n = torch.stack(torch.meshgrid(*[a[:-1] for a in axes], indexing="ij"), dim=-1).reshape(-1, 3)
    hi_n = torch.stack(torch.meshgrid(*[a[1:] for a in axes], indexing="ij"), dim=-1).reshape(-1, 3)
    bounds = torch.stack([lo + size * lo_n, lo + size * hi_n], dim=1)
    return bounds, (bounds[:, 1] - bounds[:, 0]).abs()


_ROUTE_PLANS: Dict[tuple, tuple] = {}


def _route_plan(aabb: torch.Tensor, cells: Tuple[int, int, int], device):
    """Host-side constants of one region's routing, cached: cell bounds / per-cell keep tolerance on
    the device, tol_abs = max(1e-6 * median cell diagonal, 1e-9), the kernel's host arrays."""
    a = tuple(aabb.detach().float().cpu().reshape(-1).tolist())
    key = (a, tuple(int(c) for c in cells), str(device))
    plan = _ROUTE_PLANS.get(key)
    if plan is None:
        bounds, sizes = cell_grid(aabb, cells)
        tol_abs = max(1e-6 * sizes.pow(2).sum(dim=1).sqrt().median().item(), 1e-9)
        size = (bounds[:, 1] - bounds[:, 0]).norm(dim=1)
        tol_cell = torch.maximum(1e-6 * size, torch.tensor(1e-9))
        plan = (bounds, sizes, bounds.reshape(-1).to(device), tol_cell.to(device), float(tol_abs),
                (C.c_float * 6)(*a), (C.c_int32 * 3)(*key[1]))
        if len(_ROUTE_PLANS) > 64:
            _ROUTE_PLANS.clear()
        _ROUTE_PLANS[key] = plan
    return plan


def route_rays(rays: torch.Tensor, aabb: torch.Tensor, cells: Tuple[int, int, int], alpha: float,
               policy: str = "alpha", max_steps: int = 64):
    """Per ray: selected micro-cell (int64, -1 when the ray misses the region) and a keep flag
    (the selected cell's overlap passes its tolerance) -- one HIP launch (acn_route_rays)."""
    ops.require_hip(rays, "TaskDataset routing")
    r = rays.detach().to(torch.float32).contiguous()
    dev = r.device
    bounds, sizes, cb, tc, tol_abs, a_arr, c_arr = _route_plan(aabb, cells, dev)
    N = r.shape[0]
    cid = torch.empty(N, dtype=torch.int64, device=dev)
    flags = torch.empty(N, dtype=torch.uint8, device=dev)
    hook = ops.EVENT_HOOK
    if hook is not None:
        e0 = torch.cuda.Event(enable_timing=True)
        e0.record()
    check(_lib.lib().acn_route_rays(ptr(r), N, a_arr, c_arr, ptr(cb), ptr(tc), float(alpha), tol_abs,
                                    0 if policy == "alpha" else 1, int(max_steps), ptr(cid), ptr(flags),
                                    stream_of(r)), "acn_route_rays")
    if hook is not None:
        e1 = torch.cuda.Event(enable_timing=True)
        e1.record()
        hook.append((e0, e1))
    return cid, flags, bounds, sizes


def bin_rays(cid: torch.Tensor, flags: torch.Tensor, n_cells: int):
    """Kept rays grouped by cell, ascending inside a cell (acn_bin_rays): (ray_index int32 device,
    per-cell counts list, number of region-valid rays)."""
    ops.require_hip(cid, "TaskDataset binning")
    N = int(cid.numel())
    L = _lib.lib()
    ws = torch.empty(int(L.acn_bin_rays_workspace_bytes(N, int(n_cells))), dtype=torch.uint8, device=cid.device)
    out = torch.empty(max(N, 1), dtype=torch.int32, device=cid.device)
    counts = torch.empty(n_cells + 1, dtype=torch.int64, device=cid.device)
    check(L.acn_bin_rays(ptr(cid), ptr(flags), N, int(n_cells), ptr(out), ptr(counts), ptr(ws), ws.numel(),
                         stream_of(cid)), "acn_bin_rays")
    c = counts.cpu().tolist()
    return out[: sum(c[:n_cells])], c[:n_cells], c[n_cells]


class TaskDataset(IterableDataset):
    """Micro-cell episodic dataset over a (device) ray table (task_dataset.py:29-1004): same
    constructor, attributes and episode semantics; routing on the GPU, sampling decisions drawn from
    the reference's CPU generator in the reference's order, rays gathered on the device."""

    def __init__(self, ram_ds, cell_id: int, S_target: int = 4000, Q_target: int = 2000, min_rays_cell: int = 6000,
                 image_cap: Optional[float] = None, max_images_support: Optional[int] = 8,
                 max_images_query: Optional[int] = 4, min_images_support: int = 2, min_images_query: int = 1,
                 region_bounds=None, cells: Tuple[int, int, int] = (1, 6, 6), cell_pick: str = "uniform",
                 assignment_checkpoint: float = 0.7, routing_policy: str = "alpha", image_disjoint_splits: bool = True,
                 overlap_bias_exponent: float = 0.6, debug: bool = False, seed: int = 0, bins=None):
        super().__init__()
        for attr in ("_rays", "_rgbs", "_img_indices"):
            if not hasattr(ram_ds, attr):
                raise ValueError(f"RamRaysDataset missing attribute {attr}; got type {type(ram_ds)}")
        self.rays, self.rgbs, self.imgix = ram_ds._rays, ram_ds._rgbs, ram_ds._img_indices
        self.uv = None
        self.max_images_support, self.max_images_query = max_images_support, max_images_query
        self.min_images_support, self.min_images_query = int(min_images_support), int(min_images_query)
        self.seed = int(seed)
        self.rng = torch.Generator(device=torch.device("cpu"))
        self.rng.manual_seed(self.seed)
        self.cell_id = int(cell_id)
        self.S_target, self.Q_target = int(S_target), int(Q_target)
        self.min_rays_cell = int(min_rays_cell)
        self.image_cap = image_cap
        self.region_bounds_in = region_bounds
        self.cells = tuple(int(c) for c in cells)
        self.cell_pick = cell_pick
        self.assignment_checkpoint = float(max(0.0, min(1.0, assignment_checkpoint)))
        self.routing_policy = str(routing_policy).lower()
        assert self.routing_policy in ("alpha", "dda")
        self.image_disjoint_splits = bool(image_disjoint_splits)
        self.overlap_bias_exponent = float(overlap_bias_exponent)
        self.debug = bool(debug)
        self.N_total = int(self.rays.shape[0])
        self.device = self.rays.device
        self.aabb = self._region_aabb(self.rays, region_bounds)
        self.cell_bounds, self.cell_sizes = cell_grid(self.aabb, self.cells)
        self._imgix_host = self.imgix.detach().to("cpu", torch.int64)
        if bins is None:
            bins = self._route_and_bin()
        self._build_cell_cache(bins)
        self._cursor = 0
        self.eligible_cells = [i for i, n in enumerate(self._cell_total_counts) if n >= self.min_rays_cell]
        if not self.eligible_cells:
            warnings.warn(f"[Region {self.cell_id}] No eligible cells (min_rays_cell={self.min_rays_cell}).")

    # ------------------------------------------------------------------ routing
    @staticmethod
    def _region_aabb(rays: torch.Tensor, region_bounds):
        """Given bounds, or the box of the rays' near points (task_dataset.py:229-239)."""
        if region_bounds is not None:
            return torch.tensor(region_bounds, dtype=torch.float32)
        pts = rays[:, 0:3] + rays[:, 3:6] * rays[:, 6:7]
        return torch.stack([pts.min(dim=0).values, pts.max(dim=0).values], dim=0).cpu()

    def _route_and_bin(self) -> List[torch.Tensor]:
        """Per-cell ray index lists (task_dataset.py:544-628): HIP routing + keep filter, then the
        cells ordered like the reference's ``torch.argsort`` over the region-valid rays.  That CPU
        argsort is a stable radix sort from 32768 elements on (the regime of real regions) -- done
        here by the stable counting sort acn_bin_rays -- and an unstable introsort below, whose tie
        order only the same host call reproduces, so small regions sort their cell ids on the host."""
        C_ = self.cell_bounds.shape[0]
        cid, flags, _, _ = route_rays(self.rays, self.aabb, self.cells, self.assignment_checkpoint,
                                      self.routing_policy)
        idx, counts, n_valid = bin_rays(cid, flags, C_)
        if n_valid < _RADIX_SORT_MIN:
            cid, flags = cid.cpu(), flags.cpu()
            iv = torch.nonzero((flags & 1) != 0, as_tuple=False).reshape(-1)
            order = torch.argsort(cid.index_select(0, iv))
            c, ix = cid.index_select(0, iv).index_select(0, order), iv.index_select(0, order)
            k = (flags.index_select(0, ix) & 2) != 0
            c, ix = c[k], ix[k]
            return [ix[c == j] for j in range(C_)]
        host = torch.empty(idx.numel(), dtype=torch.int32, pin_memory=True)
        host.copy_(idx)
        return list(torch.split(host, counts))

    # ------------------------------------------------------------------ cell pools
    def _build_cell_cache(self, cell_bins: List[torch.Tensor]):
        """Each cell's pool in a seeded random order (task_dataset.py:630-680); host-side index lists."""
        self._cell_flat_idx, self._cell_flat_img, self._cell_total_counts = [], [], []
        self._cell_concat_idx, self._cell_img_ids = [], []
        self._cell_img_starts, self._cell_img_lengths = [], []
        uniq = self.debug or self.image_disjoint_splits
        empty = torch.empty(0, dtype=torch.long)
        for pool in cell_bins:
            pool = pool.to("cpu", torch.int64)
            n = int(pool.numel())
            if n == 0:
                for lst in (self._cell_flat_idx, self._cell_flat_img, self._cell_concat_idx, self._cell_img_ids,
                            self._cell_img_starts, self._cell_img_lengths):
                    lst.append(empty)
                self._cell_total_counts.append(0)
                continue
            flat = pool.index_select(0, torch.randperm(n, generator=self.rng))
            img = self._imgix_host.index_select(0, flat)
            self._cell_flat_idx.append(flat)
            self._cell_flat_img.append(img)
            self._cell_concat_idx.append(flat)
            self._cell_img_ids.append(torch.unique(img) if uniq else empty)
            self._cell_img_starts.append(empty)
            self._cell_img_lengths.append(empty)
            self._cell_total_counts.append(n)

    # ------------------------------------------------------------------ sampling
    @staticmethod
    def _split_support_query(N: int, S_target: int, Q_target: int):
        """(S, Q) sizes, keeping the S:Q ratio when the cell is underfilled."""
        if N >= S_target + Q_target:
            return S_target, Q_target
        r = float(S_target) / float(Q_target)
        S = max(0, min(int(round(N * r / (1.0 + r))), N))
        return S, N - S

    @staticmethod
    def _freq_sorted_unique(img_ix_tensor: torch.Tensor) -> List[int]:
        vals, cnt = torch.unique(img_ix_tensor, return_counts=True)
        return vals[torch.argsort(cnt, descending=True)].tolist()

    def _pick_cell(self) -> Optional[int]:
        if not self.eligible_cells:
            return None
        if self.cell_pick == "sequential":
            cid = self.eligible_cells[self._cursor % len(self.eligible_cells)]
            self._cursor += 1
            return int(cid)
        return int(self.eligible_cells[torch.randint(len(self.eligible_cells), (1,), generator=self.rng).item()])

    def _shuffled(self, t: torch.Tensor, k: int) -> torch.Tensor:
        """k elements of t in a fresh generator permutation."""
        return t.index_select(0, torch.randperm(t.numel(), generator=self.rng)[:k])

    def _choose_images_for_split(self, cid: int, min_imgs: int, max_imgs: Optional[int],
                                 forbid_imgs: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Random image subset of the cell, avoiding ``forbid_imgs`` unless needed to reach the minimum."""
        imgs = torch.unique(self._cell_flat_img[cid])
        if imgs.numel() == 0:
            return imgs
        forbidden = torch.isin(imgs, forbid_imgs) if forbid_imgs is not None and forbid_imgs.numel() else None
        pool = imgs if forbidden is None else imgs[~forbidden]
        kmax = imgs.numel() if (max_imgs is None or max_imgs <= 0) else min(max_imgs, imgs.numel())
        kmin = max(0, min(min_imgs, kmax))
        if pool.numel() >= kmin:
            return self._shuffled(pool, min(kmax, pool.numel()))
        chosen = pool
        if forbidden is not None and chosen.numel() < kmin:
            borrow = imgs[forbidden]
            need = min(kmin, kmax) - chosen.numel()
            if need > 0 and borrow.numel() > 0:
                chosen = torch.cat([chosen, self._shuffled(borrow, min(need, borrow.numel()))], 0)
        if chosen.numel() > kmax:
            chosen = self._shuffled(chosen, kmax)
        return chosen

    def _sample_split_from_images(self, cid: int, target: int, images: torch.Tensor,
                                  forbid_indices: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Random rays of the cell from ``images``, ray-disjoint from ``forbid_indices``; with
        ``image_cap`` an image contributes at most ceil(cap * need) rays (the first ones in the draw)."""
        flat_idx, flat_img = self._cell_flat_idx[cid], self._cell_flat_img[cid]
        if target <= 0 or images is None or images.numel() == 0:
            return flat_idx[:0]
        m = torch.isin(flat_img, images)
        if forbid_indices is not None and forbid_indices.numel() > 0:
            m &= ~torch.isin(flat_idx, forbid_indices)
        pool_idx, pool_img = flat_idx[m], flat_img[m]
        if pool_idx.numel() == 0:
            return flat_idx[:0]
        need = min(int(target), int(pool_idx.numel()))
        order = torch.randperm(pool_idx.numel(), generator=self.rng)
        if not (self.image_cap is not None and self.image_cap > 0):
            return pool_idx.index_select(0, order[:need])
        cap = max(1, int(math.ceil(float(self.image_cap) * need)))
        # greedy in draw order == each image's first `cap` draws, then the first `need` of those
        img = pool_img.index_select(0, order)
        rank = torch.zeros_like(img)
        uimg, inv = torch.unique(img, return_inverse=True)
        srt = torch.sort(inv, stable=True)
        first = torch.zeros(uimg.numel(), dtype=torch.long)
        cnt = torch.bincount(inv, minlength=uimg.numel())
        first[1:] = torch.cumsum(cnt, 0)[:-1]
        rank[srt.indices] = torch.arange(img.numel()) - first[srt.values]
        picked = order[rank < cap][:need]
        return pool_idx.index_select(0, picked) if picked.numel() else pool_idx[:0]

    def _sample_split(self, cid: int, target: int, prefer_images: Optional[torch.Tensor] = None,
                      forbid_indices: Optional[torch.Tensor] = None) -> torch.Tensor:
        imgs = prefer_images if prefer_images is not None and prefer_images.numel() > 0 else \
            torch.unique(self._cell_flat_img[cid])
        return self._sample_split_from_images(cid, target, imgs, forbid_indices)

    def _gather(self, sel: torch.Tensor) -> Dict[str, torch.Tensor]:
        d = sel.to(self.device, non_blocking=True)
        out = {"rays": self.rays.index_select(0, d), "rgbs": self.rgbs.index_select(0, d),
               "img_indices": self.imgix.index_select(0, d), "idx": sel}
        out["img_ids"] = out["img_indices"]
        return out

    def __iter__(self):
        """Endless episodes (task_dataset.py:815-965)."""
        info = torch.utils.data.get_worker_info()
        if info is not None:
            self.rng.manual_seed(self.seed + info.id)
        if not self.eligible_cells:
            return
        while True:
            cid = self._pick_cell()
            if cid is None:
                return
            N = self._cell_total_counts[cid]
            if N < self.min_rays_cell:
                continue
            S, Q = self._split_support_query(N, self.S_target, self.Q_target)
            s_imgs = self._choose_images_for_split(cid, self.min_images_support, self.max_images_support, None)
            sel_s = self._sample_split_from_images(cid, S, s_imgs, None)
            q_imgs = self._choose_images_for_split(cid, self.min_images_query, self.max_images_query,
                                                   s_imgs if self.image_disjoint_splits else None)
            sel_q = self._sample_split_from_images(cid, Q, q_imgs, torch.unique(sel_s))
            if sel_q.numel() < Q and self.image_disjoint_splits:
                extra = self._sample_split_from_images(cid, Q - sel_q.numel(), torch.unique(self._cell_flat_img[cid]),
                                                       torch.unique(torch.cat([sel_s, sel_q], 0)))
                if extra.numel() > 0:
                    sel_q = torch.cat([sel_q, extra], 0)
            img_s = self._imgix_host.index_select(0, sel_s)
            img_q = self._imgix_host.index_select(0, sel_q)
            if self.debug:
                assert sel_s.numel() == sel_s.unique().numel() and sel_q.numel() == sel_q.unique().numel()
                assert not bool(torch.isin(sel_s, sel_q).any()), "S/Q rays are not disjoint!"
            disjoint = not (img_s.numel() and img_q.numel() and bool(torch.isin(img_s, img_q).any()))
            notes = [] if (disjoint or not self.image_disjoint_splits) else \
                ["[fallback] borrowed from support images (still ray-disjoint)"]
            metrics = {"S": float(sel_s.numel()), "Q": float(sel_q.numel()), "total_cell": float(N),
                       "num_cells": float(self.cell_bounds.shape[0]),
                       "routing_policy": 1.0 if self.routing_policy == "dda" else 0.0,
                       "alpha": float(self.assignment_checkpoint), "image_disjoint_ok": 1.0 if disjoint else 0.0}
            yield Task(support=self._gather(sel_s), query=self._gather(sel_q), cell_id=self.cell_id, block_id=cid,
                       bounds=self.cell_bounds[cid],
                       support_imgs=self._freq_sorted_unique(img_s) if self.debug else None,
                       query_imgs=self._freq_sorted_unique(img_q) if self.debug else None,
                       warnings=notes, metrics=metrics)

    def __len__(self):
        return len(self.eligible_cells)


RamRaysDataset = DeviceRaysDataset  # the reference's name (data/ram_rays_dataset.py:127)
