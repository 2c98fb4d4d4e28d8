"""Cluster creation on the GPU: scripts/create_clusters.py.

Same command line, outputs and file formats as the reference (``masks/<output>/params.pt``,
``scene_boxes.pt``/``.txt`` and one zipped bool (H, W) mask per centroid per image), with the
per-image work on the device:

* rays: acn_ray_directions + acn_rays_from_dirs (get_rays with the global SceneBox, max_bound 1e10,
  misses tagged inf) + acn_clamp_rays (the near/far override), all bit-exact;
* routing: ONE acn_voronoi_route launch per image (csrc/clusters.hip) replaces compute_voronoi_opt's
  chunked (R*S, C) distance GEMMs, the per-expert nonzero/gather/min/max loop and the host copy of
  the (N, C) mask, or compute_voronoi_orig's cdist blocks (``--orig``);
* per-expert boxes and sample counts are streamed by that launch into device buffers and reduced
  across ranks with RCCL all-reduces (MIN / MAX / SUM), as the reference does over NCCL;
* centroids (grid / k-means over the camera centres) are the reference's host torch code.

Images are split rank-strided (``np.arange(rank, n, world)``); ``torchrun`` sets RANK/WORLD_SIZE.
"""
from __future__ import annotations

import argparse
import datetime
import logging
import os
import zipfile
from pathlib import Path
from typing import Iterable, List, Optional, Tuple

import ctypes as C
import numpy as np
import torch
import torch.distributed as dist

from . import _lib, ops
from ._lib import check, ptr, stream_of
from .scene_box import SceneBox

MAX_CENTROIDS = 63


# ------------------------------------------------------------------------------------------ CLI
def parse_args(argv=None) -> argparse.Namespace:
    """create_clusters.py:97-208 -- same flags and defaults."""
    p = argparse.ArgumentParser("Create cluster masks (Voronoi routing, 2D/3D grid or kmeans) + per-expert AABBs")
    p.add_argument("--data_path", type=Path, required=True)
    p.add_argument("--output", type=Path, required=True)
    p.add_argument("--segmentation_path", type=Path, default=None)
    p.add_argument("--resume", action="store_true")
    p.add_argument("--centroid_mode", choices=["grid", "kmeans"], default="grid")
    p.add_argument("--grid_dim", nargs="+", type=int, metavar="D", required=True)
    p.add_argument("--cluster_2d", action="store_true")
    p.add_argument("--kmeans_iters", type=int, default=50)
    p.add_argument("--kmeans_init", choices=["kmeans++", "random"], default="kmeans++")
    p.add_argument("--kmeans_seed", type=int, default=0)
    p.add_argument("--kmeans_weight_by_pixels", action="store_true")
    p.add_argument("--boundary_margin", type=float, default=1.0)
    p.add_argument("--ray_samples", type=int, default=256)
    p.add_argument("--center_pixels", action="store_true")
    p.add_argument("--orig", action="store_true")
    p.add_argument("--ray_chunk_size", type=int, default=256 * 1024)
    p.add_argument("--sample_chunk_size", type=int, default=512 * 1024 * 1024)
    p.add_argument("--fp16", action="store_true")
    p.add_argument("--scene_scale", type=float, default=1.0)
    p.add_argument("--altitude_range", nargs=2, type=float, default=None)
    p.add_argument("--near", type=float, default=None)
    p.add_argument("--far", type=float, default=None)
    p.add_argument("--altitude_pad", type=float, default=10.0)
    p.add_argument("--box_margin", type=float, default=0.0)
    return p.parse_args(argv)


def _log(rank: int, *msg) -> None:
    if rank == 0:
        logging.info(" ".join(str(m) for m in msg))


def _init_distributed(out_dir: Path, resume: bool) -> Tuple[int, int, torch.device]:
    """One process per GPU over RCCL when launched by torchrun (create_clusters.py:224-238)."""
    if "RANK" in os.environ and "WORLD_SIZE" in os.environ:
        local = int(os.environ.get("LOCAL_RANK", "0"))
        torch.cuda.set_device(local)
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group(backend="nccl", timeout=datetime.timedelta(hours=24),
                                device_id=torch.device("cuda", local))
        rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
        if rank == 0:
            out_dir.mkdir(parents=True, exist_ok=resume)
        dist.barrier()
        return rank, world, torch.device("cuda", local)
    out_dir.mkdir(parents=True, exist_ok=resume)
    if not torch.cuda.is_available():
        raise RuntimeError("create_clusters: the HIP routing kernel needs a GPU (no CPU path)")
    return 0, 1, torch.device("cuda", torch.cuda.current_device())


def _meta_list(ds_root: Path, split: str) -> List[Path]:
    return sorted((ds_root / split / "metadata").glob("*.pt"))


def _save_zip_tensor(path: Path, tensor: torch.Tensor) -> None:
    """Zipped torch.save, inner name = file name (create_clusters.py:245-249)."""
    path.parent.mkdir(parents=True, exist_ok=True)
    with zipfile.ZipFile(path, "w", compression=zipfile.ZIP_DEFLATED) as zf, zf.open(path.name, "w") as f:
        torch.save(tensor, f)


def _read_zip_tensor(path: Path, inner: Optional[str] = None):
    with zipfile.ZipFile(path, "r") as zf:
        name = inner if inner in zf.namelist() else zf.namelist()[0]
        with zf.open(name, "r") as f:
            return torch.load(f, map_location="cpu", weights_only=True)


def _zip_load_ok(path: Path, inner: Optional[str] = None) -> bool:
    if not path.exists():
        return False
    try:
        _read_zip_tensor(path, inner or path.name)
        return True
    except Exception:
        return False


def all_ok_for_image(K: int, out_dir: Path, filename: str) -> bool:
    return all(_zip_load_ok(out_dir / str(cid) / filename, filename) for cid in range(K))


def _read_zip_mask(zip_path: Path) -> Optional[torch.Tensor]:
    if not zip_path.exists():
        return None
    try:
        return _read_zip_tensor(zip_path)
    except Exception:
        return None


def _cam_weights(meta_paths: Iterable[Path]) -> Optional[torch.Tensor]:
    ws = []
    for p in meta_paths:
        md = torch.load(p, map_location="cpu", weights_only=True)
        ws.append(int(md["H"]) * int(md["W"]))
    return torch.tensor(ws, dtype=torch.float32) if ws else None


# ------------------------------------------------------------------------------------ centroids
def _grid_centroids(cam_pos: torch.Tensor, gx: int, gy: int, gz: int, cluster_2d: bool) -> torch.Tensor:
    """Tile / cube centres over the camera bounding box (create_clusters.py:298-323)."""
    if cam_pos.numel() == 0:
        return torch.zeros(((gy * gz) if cluster_2d else (gx * gy * gz), 3), dtype=torch.float32)
    lo, hi = cam_pos.min(0).values, cam_pos.max(0).values
    if cluster_2d:
        Y = lo[1] + (torch.arange(gy) + 0.5) * ((hi[1] - lo[1]) / gy)
        Z = lo[2] + (torch.arange(gz) + 0.5) * ((hi[2] - lo[2]) / gz)
        YY, ZZ = torch.meshgrid(Y, Z, indexing="ij")
        return torch.stack((torch.full_like(YY, (lo[0] + hi[0]) * 0.5), YY, ZZ), -1).reshape(-1, 3)
    axes = [lo[a] + (torch.arange(g) + 0.5) * ((hi[a] - lo[a]) / max(g, 1)) for a, g in enumerate((gx, gy, gz))]
    return torch.stack(torch.meshgrid(*axes, indexing="ij"), -1).reshape(-1, 3)


def _kmeans_init(points: torch.Tensor, K: int, seed: int, method: str, weights: Optional[torch.Tensor]):
    """k-means++ (optionally pixel-weighted) or random seeds (create_clusters.py:326-352)."""
    g = torch.Generator(device="cpu").manual_seed(seed)
    if method == "random":
        return points[torch.randperm(points.size(0), generator=g)[:K]].clone()
    cen = torch.empty(K, points.size(1), dtype=points.dtype)
    if weights is None:
        cen[0] = points[torch.randint(points.size(0), (1,), generator=g)]
    else:
        cen[0] = points[torch.multinomial((weights / weights.sum()).cpu(), 1, generator=g)]
    for k in range(1, K):
        d2 = torch.cdist(points, cen[:k]).min(1).values ** 2
        pr = (d2 * (weights if weights is not None else 1.0)).clamp_min_(1e-12)
        cen[k] = points[torch.multinomial(pr / pr.sum(), 1, generator=g)]
    return cen


def _run_kmeans(points: torch.Tensor, K: int, iters: int, init: str, seed: int, weights: Optional[torch.Tensor]):
    """Lloyd iterations; an empty cluster jumps to its farthest point (create_clusters.py:355-377)."""
    cen = _kmeans_init(points, K, seed, init, weights)
    w = weights if weights is not None else torch.ones(points.size(0), dtype=points.dtype)
    for _ in range(max(1, iters)):
        D = torch.cdist(points, cen)
        a = D.argmin(1)
        for k in range(K):
            m = a == k
            cen[k] = points[D[:, k].argmax()] if not m.any() else (w[m][:, None] * points[m]).sum(0) / w[m].sum()
    return cen


# ------------------------------------------------------------------------------------ routing
def voronoi_route(rays: torch.Tensor, ray_samples: int, centroids: torch.Tensor, cluster_2d: bool,
                  boundary_margin: float, orig: bool = False, update_aabbs: bool = False, mins_out=None,
                  maxs_out=None, counts_out=None, nan_out=None) -> torch.Tensor:
    """One acn_voronoi_route launch: (N,) uint64 centroid bits per ray (as int64 storage).  With
    update_aabbs (opt modes) mins_out / maxs_out (C,3) f32, counts_out (C) int64 and nan_out (C)
    int32 device tensors are updated in place."""
    ops.require_hip(rays, "create_clusters routing")
    r = rays.detach().to(torch.float32).reshape(-1, 8).contiguous()
    cents = centroids.detach().float().cpu().reshape(-1, 3).contiguous()
    Cn = cents.shape[0]
    if Cn > MAX_CENTROIDS:
        raise ValueError(f"at most {MAX_CENTROIDS} centroids per launch, got {Cn}")
    bits = torch.empty(r.shape[0], dtype=torch.int64, device=r.device)
    upd = bool(update_aabbs) and not orig
    if upd:
        for t, dt in ((mins_out, torch.float32), (maxs_out, torch.float32), (counts_out, torch.int64),
                      (nan_out, torch.int32)):
            if t is None or t.device != r.device or t.dtype != dt or not t.is_contiguous():
                raise ValueError("update_aabbs needs contiguous device mins/maxs (f32), counts (int64), nan (int32)")
    c_arr = (C.c_float * (3 * Cn))(*cents.view(-1).tolist())
    hook = ops.EVENT_HOOK
    if hook is not None:
        e0 = torch.cuda.Event(enable_timing=True)
        e0.record()
    check(_lib.lib().acn_voronoi_route(ptr(r), r.shape[0], int(ray_samples), c_arr, Cn, int(bool(cluster_2d)),
                                       float(boundary_margin), int(bool(orig)), int(upd), ptr(bits),
                                       ptr(mins_out) if upd else None, ptr(maxs_out) if upd else None,
                                       ptr(counts_out) if upd else None, ptr(nan_out) if upd else None,
                                       stream_of(r)), "acn_voronoi_route")
    if hook is not None:
        e1 = torch.cuda.Event(enable_timing=True)
        e1.record()
        hook.append((e0, e1))
    return bits


def bits_to_masks(bits: torch.Tensor, C_: int) -> torch.Tensor:
    """(N,) centroid bits -> (N, C) bool (on the bits' device)."""
    sh = torch.arange(C_, device=bits.device, dtype=torch.int64)
    return ((bits.view(-1, 1) >> sh.view(1, -1)) & 1).bool()


def compute_voronoi_opt(rays: torch.Tensor, *, ray_samples: int, ray_chunk_size: int = 0, sample_chunk_size: int = 0,
                        centroids: torch.Tensor, cluster_2d: bool, device=None, boundary_margin: float,
                        fp16: bool = False, update_aabbs: bool = False, mins_out=None, maxs_out=None,
                        counts_out=None) -> torch.Tensor:
    """create_clusters.py:386-556: (N, C) bool mask on the CPU; the chunk sizes are accepted and not
    needed (nothing of size N*S*C is formed); fp16 is ignored (fp32 routing).  AABBs stream into
    mins_out / maxs_out / counts_out (device, updated in place) when update_aabbs."""
    dev = torch.device(device) if device is not None else rays.device
    r = rays.to(dev)
    Cn = centroids.shape[0]
    nan = torch.zeros(Cn, dtype=torch.int32, device=dev) if update_aabbs else None
    bits = voronoi_route(r, ray_samples, centroids, cluster_2d, boundary_margin, False, update_aabbs, mins_out,
                         maxs_out, counts_out, nan)
    if update_aabbs and bool(nan.any()):
        nf = nan.bool()
        mins_out[nf] = float("nan")
        maxs_out[nf] = float("nan")
    return bits_to_masks(bits, Cn).cpu()


def compute_voronoi_orig(rays: torch.Tensor, *, ray_samples: int, ray_chunk_size: int = 0, sample_chunk_size: int = 0,
                         centroids: torch.Tensor, cluster_2d: bool, device=None, boundary_margin: float,
                         eps: float = 1e-8) -> torch.Tensor:
    """create_clusters.py:559-634 (cdist ratio rule, no AABB streaming): (N, C) bool on the CPU."""
    if eps != 1e-8:
        raise ValueError("the kernel implements the reference's eps = 1e-8")
    dev = torch.device(device) if device is not None else rays.device
    bits = voronoi_route(rays.to(dev), ray_samples, centroids, cluster_2d, boundary_margin, orig=True)
    return bits_to_masks(bits, centroids.shape[0]).cpu()


# ------------------------------------------------------------------------------------ scene
def global_scene_box(coord: dict, scene_scale: float, altitude_range=None, altitude_pad: float = 10.0):
    """Global SceneBox of main() (create_clusters.py:650-700): the altitude band in normalised DRB x
    (from --altitude_range or coordinates.pt) x [-scale, scale]^2, padded by altitude_pad metres in x."""
    pose_scale = float(coord.get("pose_scale_factor", 1.0))
    origin_x = float(coord.get("origin_drb", [0.0, 0.0, 0.0])[0])
    if altitude_range is not None:
        lo_m, hi_m = map(float, altitude_range)
    elif "altitude_range_enu" in coord:
        lo_m, hi_m = map(float, coord["altitude_range_enu"])
    else:
        raise ValueError("create_clusters needs --altitude_range or coordinates.pt altitude_range_enu "
                         "(the reference's box has no x extent without it)")
    if lo_m > hi_m:
        lo_m, hi_m = hi_m, lo_m
    xa, xb = -hi_m, -lo_m
    if xa > xb:
        xa, xb = xb, xa
    aabb = torch.tensor([[(xa - origin_x) / pose_scale, -scene_scale, -scene_scale],
                         [(xb - origin_x) / pose_scale, scene_scale, scene_scale]], dtype=torch.float32)
    box = SceneBox.from_bound(aabb=aabb).expand(torch.tensor([[altitude_pad / pose_scale, 0, 0]],
                                                             dtype=torch.float32))
    return box, pose_scale


def image_rays(md: dict, center_pixels: bool, box: SceneBox, near_far_override, device):
    """get_ray_directions + get_rays(scene_box, max_bound 1e10, invalid inf) + clamp_rays_near_far
    (create_clusters.py:790-803) on the device: (H*W, 8) rays and (H*W,) validity."""
    H, W = int(md["H"]), int(md["W"])
    fx, fy, cx, cy = [float(v) for v in md["intrinsics"]]
    dirs = ops.ray_directions(H, W, fx, fy, cx, cy, center_pixels, device)
    rays = ops.rays_from_dirs(dirs, md["c2w"].float(), box.aabb, eps=1e-8, max_bound=1e10,
                              invalid_value=float("inf"))
    return ops.clamp_rays(rays, near_far_override)


def final_boxes(mins, maxs, cnts, cents, aabb_global, box_margin: float = 0.0, pose_scale: float = 1.0):
    """Clamp to the global box, epsilon boxes around the centroids of empty experts, optional dilation,
    x extent = the global altitude band for every expert (create_clusters.py:930-962)."""
    lo, hi = aabb_global[0], aabb_global[1]
    mins, maxs = torch.maximum(mins, lo), torch.minimum(maxs, hi)
    empties = cnts == 0
    if empties.any():
        eps = torch.clamp((hi - lo).abs() * 1e-6, min=1e-7)
        cc = torch.minimum(torch.maximum(cents, lo), hi)
        mins[empties] = torch.maximum(cc[empties] - eps, lo)
        maxs[empties] = torch.minimum(cc[empties] + eps, hi)
    if box_margin and box_margin > 0.0:
        m = float(box_margin) / pose_scale
        mins, maxs = torch.maximum(mins - m, lo), torch.minimum(maxs + m, hi)
    mins[:, 0] = lo[0]
    maxs[:, 0] = hi[0]
    return mins, maxs


def make_centroids(h, metas: List[Path]) -> Tuple[torch.Tensor, Tuple[int, int, int]]:
    dims = list(map(int, h.grid_dim))
    if h.cluster_2d:
        if len(dims) != 2:
            raise ValueError("For cluster_2d=True use --grid_dim GY GZ.")
        gx, gy, gz = 1, dims[0], dims[1]
    elif len(dims) == 2:
        gx, gy, gz = 1, dims[0], dims[1]
    elif len(dims) == 3:
        gx, gy, gz = dims
    else:
        raise ValueError("For 3D grid use --grid_dim GX GY GZ.")
    K = gx * gy * gz
    cams = torch.stack([torch.load(p, map_location="cpu", weights_only=True)["c2w"] for p in metas]
                       ).to(torch.float32)[..., :3, 3]
    wts = _cam_weights(metas) if h.kmeans_weight_by_pixels else None
    if h.centroid_mode == "grid":
        return _grid_centroids(cams, gx, gy, gz, h.cluster_2d), (gx, gy, gz)
    if h.cluster_2d:
        yz = _run_kmeans(cams[:, 1:].cpu(), K, h.kmeans_iters, h.kmeans_init, h.kmeans_seed, wts)
        xm = (cams[:, 0].min() + cams[:, 0].max()) * 0.5
        return torch.cat([torch.full((K, 1), float(xm)), yz], dim=1), (gx, gy, gz)
    return _run_kmeans(cams.cpu(), K, h.kmeans_iters, h.kmeans_init, h.kmeans_seed, wts), (gx, gy, gz)


def _all_reduce(t: torch.Tensor, op, group=None):
    if dist.is_initialized():
        dist.all_reduce(t, op=op, group=group)
    return t


def reduce_boxes(mins, maxs, cnts, nan, group=None):
    """Cross-rank MIN / MAX / SUM of the streamed boxes (create_clusters.py:924-928); an expert with a
    NaN sample anywhere ends NaN (the reference's torch.minimum/maximum propagate it)."""
    _all_reduce(mins, dist.ReduceOp.MIN, group)
    _all_reduce(maxs, dist.ReduceOp.MAX, group)
    _all_reduce(cnts, dist.ReduceOp.SUM, group)
    _all_reduce(nan, dist.ReduceOp.MAX, group)
    nf = nan.bool()
    if nf.any():
        mins[nf] = float("nan")
        maxs[nf] = float("nan")
    return mins, maxs, cnts


@torch.inference_mode()
def main(h: argparse.Namespace) -> dict:
    """create_clusters.py:642-1015.  Returns the saved scene-box dict (rank 0) for callers and tests."""
    out = h.data_path / "masks" / h.output
    rank, world, device = _init_distributed(out, h.resume)
    logging.basicConfig(level=(logging.INFO if rank == 0 else logging.ERROR), format="%(message)s")
    ds = h.data_path
    coord = torch.load(ds / "coordinates.pt", map_location="cpu", weights_only=True)
    global_box, pose_scale = global_scene_box(coord, h.scene_scale, h.altitude_range, h.altitude_pad)
    aabb_global = global_box.aabb.detach().to(torch.float32)
    _log(rank, f"Global SceneBox: {global_box}")
    all_meta = _meta_list(ds, "train") + _meta_list(ds, "val")
    if not all_meta:
        raise RuntimeError(f"No metadata found in {ds}/{{train,val}}/metadata")
    cents, (gx, gy, gz) = make_centroids(h, all_meta)
    Cn = cents.size(0)
    if rank == 0:
        torch.save({"format_version": 3, "centroid_mode": h.centroid_mode, "centroids": cents.detach().cpu(),
                    "grid_dim": (gx, gy, gz), "cluster_2d": bool(h.cluster_2d),
                    "boundary_margin": float(h.boundary_margin), "ray_samples": int(h.ray_samples),
                    "aabb_global": aabb_global.cpu().contiguous(), "scene_scale": float(h.scene_scale),
                    "near_far_override_m": ((float(h.near) if h.near is not None else None),
                                            (float(h.far) if h.far is not None else None))}, out / "params.pt")
    if dist.is_initialized():
        dist.barrier()
    cents = cents.to(torch.float32)
    nf_override = ((float(h.near) / pose_scale) if h.near is not None else None,
                   (float(h.far) / pose_scale) if h.far is not None else None)
    box_dev = SceneBox(aabb=aabb_global.to(device))
    mins = torch.full((Cn, 3), float("inf"), dtype=torch.float32, device=device)
    maxs = torch.full((Cn, 3), float("-inf"), dtype=torch.float32, device=device)
    cnts = torch.zeros(Cn, dtype=torch.int64, device=device)
    nan = torch.zeros(Cn, dtype=torch.int32, device=device)
    for split in ("train", "val"):
        meta = _meta_list(ds, split)
        _log(rank, f"[{split}] images: {len(meta)} | rank {rank}/{world}")
        _log(rank, f"[{split}] boundary_margin={h.boundary_margin}")
        tot_pix = torch.zeros((), dtype=torch.int64, device=device)
        pix_per_cell = torch.zeros(Cn, dtype=torch.int64, device=device)
        imgs_with_pix = torch.zeros(Cn, dtype=torch.int64, device=device)
        rays_total = torch.zeros((), dtype=torch.int64, device=device)
        rays_hit = torch.zeros((), dtype=torch.int64, device=device)
        for i in np.arange(rank, len(meta), world):
            mp = meta[i]
            fname = mp.stem + ".pt"
            if h.resume and all_ok_for_image(Cn, out, fname):
                continue
            md = torch.load(mp, map_location="cpu", weights_only=True)
            H, W = int(md["H"]), int(md["W"])
            rays, valid = image_rays(md, h.center_pixels, box_dev, nf_override, device)
            rays_total += H * W
            rays_hit += valid.sum()
            bits = voronoi_route(rays, h.ray_samples, cents, h.cluster_2d, h.boundary_margin, orig=h.orig,
                                 update_aabbs=not h.orig, mins_out=mins, maxs_out=maxs, counts_out=cnts, nan_out=nan)
            masks = bits_to_masks(bits, Cn) & valid.view(-1, 1)
            if h.segmentation_path:
                seg = _read_zip_mask(Path(h.segmentation_path) / fname)
                if seg is not None:
                    masks &= seg.view(-1, 1).bool().to(device)
            per = masks.sum(0)
            pix_per_cell += per
            imgs_with_pix += (per > 0).to(torch.int64)
            host = masks.view(H, W, Cn).cpu()
            for cid in range(Cn):
                _save_zip_tensor(out / f"{cid}" / fname, host[..., cid].contiguous())
            tot_pix += H * W
        if dist.is_initialized():
            dist.barrier()
            for t in (tot_pix, pix_per_cell, imgs_with_pix, rays_total, rays_hit):
                dist.all_reduce(t, op=dist.ReduceOp.SUM)
        if rank == 0:
            total = int(tot_pix.item())
            pct = (pix_per_cell.double() / max(1, total) * 100.0).tolist()
            rt = int(rays_total.item())
            _log(rank, f"[{split}] SceneBox ray coverage: {int(rays_hit.item()):,} / {rt:,} "
                       f"({(float(rays_hit.item()) / max(1, rt) * 100.0):.3f}%)")
            _log(rank, f"[{split}] total_pixels={total:,}")
            _log(rank, f"[{split}] pixels_per_centroid={[int(x) for x in pix_per_cell.cpu().tolist()]}")
            _log(rank, f"[{split}] coverage_pct_per_centroid={[round(x, 4) for x in pct]}")
            _log(rank, f"[{split}] images_with_pixels_per_centroid={[int(x) for x in imgs_with_pix.cpu().tolist()]}")
    if dist.is_initialized():
        dist.barrier()
    mins, maxs, cnts = reduce_boxes(mins, maxs, cnts, nan)
    g = aabb_global.to(device)
    mins, maxs = final_boxes(mins, maxs, cnts, cents.to(device), g, getattr(h, "box_margin", 0.0), pose_scale)
    saved = {"format_version": 3, "aabb_global": aabb_global.cpu(), "mins": mins.detach().cpu(),
             "maxs": maxs.detach().cpu(), "counts": cnts.detach().cpu(), "centroids": cents.detach().cpu(),
             "grid_dim": (gx, gy, gz), "cluster_2d": bool(h.cluster_2d), "boundary_margin": float(h.boundary_margin),
             "ray_samples": int(h.ray_samples), "scene_scale": float(h.scene_scale)}
    if rank == 0:
        torch.save(saved, out / "scene_boxes.pt")
        gmin, gmax = saved["aabb_global"][0].tolist(), saved["aabb_global"][1].tolist()
        lines = ["==== GLOBAL ====", f"global.min = {np.round(gmin, 6).tolist()}",
                 f"global.max = {np.round(gmax, 6).tolist()}", "", "==== PER-EXPERT LOCAL BOXES (normalized DRB) ===="]
        for cid in range(Cn):
            mn = np.round(saved["mins"][cid].tolist(), 6).tolist()
            mx = np.round(saved["maxs"][cid].tolist(), 6).tolist()
            _log(rank, f"[AABB] expert={cid:03d} mins={mn} maxs={mx}")
            cen = np.round(saved["centroids"][cid].tolist(), 6).tolist()
            lines.append(f"[{cid:03d}] count={int(saved['counts'][cid]):9d}  centroid={cen}  min={mn}  max={mx}")
        (out / "scene_boxes.txt").write_text("\n".join(lines))
        _log(rank, "==== LOCAL SCENEBOX SUMMARY ====")
        _log(rank, f"Global AABB min={gmin}, max={gmax}")
        _log(rank, f"Experts with samples: {int((saved['counts'] > 0).sum().item())}/{Cn}")
    _log(rank, f"Done. Masks saved to: {out}")
    if dist.is_initialized():
        dist.destroy_process_group()
    return saved


if __name__ == "__main__":
    main(parse_args())
