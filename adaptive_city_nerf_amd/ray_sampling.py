"""Ray generation (reference interface: nerfs/ray_sampling.py:10-176) on HIP kernels.

get_ray_directions / get_rays / clamp_rays_near_far keep the reference's signatures and output
layouts ((H,W,3) dirs; (H,W,8) or (N,8) packed rays [o, d, near, far]); the arithmetic matches
the reference's CPU ops (tests/test_gpu_kernels.py::test_get_rays_vs_reference).
"""
from __future__ import annotations

from typing import Optional, Tuple

import torch
from torch import Tensor

from . import ops
from .scene_box import SceneBox


def _rays_cam_to_world(dirs_cam: Tensor, c2w: Tensor) -> Tuple[Tensor, Tensor]:
    """Camera-frame directions -> world-frame origins & directions (ray_sampling.py:10-24)."""
    rays = ops.rays_from_dirs(dirs_cam, c2w, None)
    shape = dirs_cam.shape
    return rays[:, :3].reshape(*shape), rays[:, 3:6].reshape(*shape)


def pack_rays(rays_o: Tensor, rays_d: Tensor, near: Tensor, far: Tensor) -> Tensor:
    return torch.cat([rays_o, rays_d, near, far], dim=-1)


def unpack_rays(rays: Tensor) -> Tuple[Tensor, Tensor, Tensor, Tensor]:
    assert rays.shape[-1] == 8, "packed rays must be (..., 8)"
    flat = rays.view(-1, 8).contiguous()
    return flat[:, :3], flat[:, 3:6], flat[:, 6:7], flat[:, 7:8]


def get_rays(directions: Tensor, c2w: Tensor, scene_box: Optional[SceneBox] = None, near: Optional[float] = None,
             far: Optional[float] = None, *, aabb_max_bound: float = 1e10, aabb_invalid_value: float = 1e10) -> Tensor:
    """(H,W,3) -> (H,W,8) or (N,3) -> (N,8) rays [o, d, near, far] (ray_sampling.py:50-108)."""
    if directions.ndim == 2 and directions.shape[1] == 3:
        out_shape = (directions.shape[0], 8)
    elif directions.ndim == 3 and directions.shape[-1] == 3:
        out_shape = (*directions.shape[:2], 8)
    else:
        raise ValueError(f"directions must be (H, W, 3) or (N, 3), got {tuple(directions.shape)}")
    if scene_box is None and (near is None or far is None):
        raise ValueError("Provide near/far when scene_box is None")
    rays = ops.rays_from_dirs(directions, c2w, None if scene_box is None else scene_box.aabb,
                              near_c=float(near or 0.0), far_c=float(far or 0.0), eps=1e-8,
                              max_bound=aabb_max_bound, invalid_value=aabb_invalid_value)
    return rays.view(*out_shape)


def get_ray_directions(H: int, W: int, fx: float, fy: float, cx: float, cy: float, center_pixels: bool,
                       device: torch.device) -> Tensor:
    """Unit camera-frame (RUB) directions (H, W, 3) for pinhole intrinsics (ray_sampling.py:111-136)."""
    return ops.ray_directions(H, W, fx, fy, cx, cy, center_pixels, device)


@torch.no_grad()
def clamp_rays_near_far(rays: Tensor, near_far_override: Optional[Tuple[Optional[float], Optional[float]]], *,
                        eps: float = 1e-6, invalid_value: float = float("inf")) -> Tuple[Tensor, Tensor]:
    """(rays', valid): optional near/far overrides; invalid rays get near=far=invalid_value
    (ray_sampling.py:139-176).  With override None the input is returned unchanged."""
    return ops.clamp_rays(rays, near_far_override, eps=eps, invalid_value=invalid_value)
