"""SceneBox (reference interface: nerfs/scene_box.py:10-217, AABB part).

The slab test ``ray_aabb_intersect`` runs on the HIP kernel (acn_ray_aabb) for device tensors;
the remaining helpers are small tensor utilities with the reference's semantics.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Tuple, Union

import torch
from torch import Tensor

from . import ops


@dataclass
class SceneBox:
    """AABB stored as (2, 3): [min, max]."""

    aabb: Tensor

    @property
    def min(self) -> Tensor:
        return self.aabb[0]

    @property
    def max(self) -> Tensor:
        return self.aabb[1]

    @property
    def center(self) -> Tensor:
        return (self.aabb[0] + self.aabb[1]) * 0.5

    @property
    def extent(self) -> Tensor:
        return self.aabb[1] - self.aabb[0]

    def to(self, dev) -> "SceneBox":
        dev = torch.device(dev) if isinstance(dev, str) else dev
        return SceneBox(aabb=self.aabb.to(dev))

    def __repr__(self) -> str:
        mn = ", ".join(f"{x:.3f}" for x in self.min.cpu().tolist())
        mx = ", ".join(f"{x:.3f}" for x in self.max.cpu().tolist())
        return f"SceneBox (min=[{mn}], max=[{mx}], diag={self.get_diagonal_length().item():.3f})"

    def ray_aabb_intersect(self, origins: Tensor, directions: Tensor, eps: float = 1e-8, max_bound: float = 1e10,
                           invalid_value: float = 1e10) -> Tuple[Tensor, Tensor]:
        """Slab test, t clamped to [0, max_bound], misses tagged invalid_value (scene_box.py:45-107)."""
        assert self.aabb.shape == (2, 3), "aabb must be (2,3)"
        out_dev = origins.device
        tmin, tmax = ops.ray_aabb(origins if origins.is_cuda else origins.cuda(), directions, self.aabb, eps,
                                  max_bound, invalid_value)
        return tmin.to(out_dev), tmax.to(out_dev)

    def within(self, pts: Tensor, inclusive: bool = False) -> Tensor:
        if inclusive:
            return (pts >= self.aabb[0]).all(dim=-1) & (pts <= self.aabb[1]).all(dim=-1)
        return (pts > self.aabb[0]).all(dim=-1) & (pts < self.aabb[1]).all(dim=-1)

    def get_diagonal_length(self) -> Tensor:
        return torch.linalg.norm(self.aabb[1] - self.aabb[0])

    def get_centered_and_scaled_scene_box(self, scale_factor: Union[float, Tensor] = 1.0) -> "SceneBox":
        return SceneBox(aabb=(self.aabb - self.center) * scale_factor)

    @staticmethod
    def get_normalized_positions(positions: Tensor, aabb: Tensor) -> Tensor:
        return (positions - aabb[0]) / (aabb[1] - aabb[0])

    @staticmethod
    def from_camera_poses(poses: Tensor, scale_factor: float) -> "SceneBox":
        xyzs = poses[..., :3, -1]
        return SceneBox(aabb=torch.stack([torch.min(xyzs, dim=0)[0], torch.max(xyzs, dim=0)[0]]) * scale_factor)

    @staticmethod
    def from_bound(aabb: Tensor) -> "SceneBox":
        """An explicit (2, 3) AABB (scene_box.py:148-160)."""
        assert isinstance(aabb, torch.Tensor), "aabb must be a torch.Tensor"
        assert aabb.shape == (2, 3), f"Expected (2,3) AABB, got {tuple(aabb.shape)}"
        return SceneBox(aabb=aabb)

    def expand(self, pad) -> "SceneBox":
        """Absolute padding (scene_box.py:162-205): scalar, per-axis (3,)/(1,3), or (2,3) [min side, max side]."""
        p = torch.as_tensor(pad, dtype=self.aabb.dtype, device=self.aabb.device)
        if p.ndim == 0:
            lo = hi = p.expand(3)
        elif tuple(p.shape) in ((3,), (1, 3)):
            lo = hi = p.view(-1, 3)[-1]
        elif tuple(p.shape) == (2, 3):
            lo, hi = p[0], p[1]
        else:
            raise ValueError(f"pad must be scalar, (3,), (1,3), or (2,3); got shape {tuple(p.shape)}")
        mn, mx = self.aabb[0] - lo, self.aabb[1] + hi
        if not torch.all(mn < mx):
            raise ValueError(f"expand produced invalid AABB: min {mn} not < max {mx}")
        return SceneBox(aabb=torch.stack([mn, mx], dim=0))

    def union(self, other: "SceneBox") -> "SceneBox":
        return SceneBox(aabb=torch.stack([torch.minimum(self.aabb[0], other.aabb[0]),
                                          torch.maximum(self.aabb[1], other.aabb[1])], dim=0))

    @staticmethod
    def reduce_union(aabbs: Tensor) -> "SceneBox":
        return SceneBox(aabb=torch.stack([aabbs[:, 0, :].min(dim=0).values, aabbs[:, 1, :].max(dim=0).values], dim=0))
