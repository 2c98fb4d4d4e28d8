"""The nerfacc 0.5.3 surface the reference's occupancy renderer uses, on MI355X HIP kernels.

The reference imports ``nerfacc`` (``from nerfacc import OccGridEstimator`` in
models/inr/meta_ngp.py:6; ``nerfacc.pack_info`` / ``render_weight_from_density`` /
``accumulate_along_rays`` in nerfs/ray_rendering.py:452-462, :540-552).  nerfacc is a third-party
CUDA extension, not vendored in the reference; this module restates its
published 0.5.3 behaviour with the same names, arguments and buffers so the reference's call sites
read unchanged:

* ``OccGridEstimator(roi_aabb, resolution=128, levels=1)``: buffers ``resolution`` (int32 [3]),
  ``aabbs`` (levels, 6), ``occs`` (levels * R^3), ``binaries`` (levels, R, R, R) bool -- the
  state-dict keys of a nerfacc checkpoint; ``sampling``, ``update_every_n_steps``,
  ``mark_invisible_cells``.  Marching runs on the HIP traversal kernel over a 1-bit-per-cell copy
  of ``binaries`` (re-derived whenever the buffer changes).
* ``pack_info``, ``render_transmittance_from_density``,
  ``render_weight_from_density``, ``render_visibility_from_density``, ``accumulate_along_rays``:
  packed (ray-major) sample arrays; weights and accumulation are HIP segmented scans / sums with
  HIP backward kernels behind autograd Functions.

Parity with nerfacc itself is UNPINNED (no nerfacc code or fixture exists in this environment); the
kernels are checked bit for bit (traversal) / within tolerance (compositing) against the oracle's
restatement (oracle/occ_oracle.c, oracle/occ_ref.py), and the reference's glue around nerfacc is
pinned by tests/golden/occ_*.npz.
"""
from __future__ import annotations

from typing import Callable, List, Optional, Tuple

import torch
import torch.nn as nn
from torch import Tensor

from . import occ_ops
from ._lib import AcnError

__all__ = ["OccGridEstimator", "ray_aabb_intersect", "traverse_grids", "pack_info",
           "render_transmittance_from_density", "render_weight_from_density", "render_visibility_from_density",
           "accumulate_along_rays"]


# ----------------------------------------------------------------------------------------------
def pack_info(ray_indices: Tensor, n_rays: Optional[int] = None) -> Tensor:
    """(n_rays, 2) [chunk_starts, chunk_cnts] of a ray-sorted sample array (nerfacc.pack_info)."""
    assert ray_indices.dim() == 1, "ray_indices must be a 1D tensor"
    if n_rays is None:
        n_rays = int(ray_indices.max().item()) + 1 if ray_indices.numel() else 0
    cnts = torch.bincount(ray_indices.long(), minlength=n_rays)[:n_rays] if ray_indices.numel() else \
        torch.zeros(n_rays, dtype=torch.long, device=ray_indices.device)
    starts = torch.cumsum(cnts, 0) - cnts
    return torch.stack([starts, cnts], -1)


def _packed(packed_info: Optional[Tensor], ray_indices: Optional[Tensor], n_rays: Optional[int], M: int, device):
    if packed_info is not None:
        return packed_info[:, 0].contiguous(), packed_info[:, 1].contiguous()
    if ray_indices is not None:
        pi = pack_info(ray_indices, n_rays)
        return pi[:, 0].contiguous(), pi[:, 1].contiguous()
    # a single ray holding every sample (nerfacc's batched-without-packing case is not used by the reference)
    return (torch.zeros(1, dtype=torch.long, device=device), torch.full((1,), M, dtype=torch.long, device=device))


class _PackedWeightsFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, sigmas, t_starts, t_ends, starts, counts):
        w, tr, al = occ_ops.packed_weights(sigmas, t_starts, t_ends, starts, counts)
        ctx.save_for_backward(sigmas, t_starts, t_ends, w, tr, al, starts, counts)
        return w, tr, al

    @staticmethod
    def backward(ctx, g_w, g_tr, g_al):
        sigmas, t0, t1, w, tr, al, starts, counts = ctx.saved_tensors
        gs = occ_ops.packed_weights_bwd(sigmas, t0, t1, w, tr, al, g_w, g_tr, g_al, starts, counts)
        return gs.view_as(sigmas), None, None, None, None


def render_transmittance_from_density(t_starts: Tensor, t_ends: Tensor, sigmas: Tensor,
                                      packed_info: Optional[Tensor] = None, ray_indices: Optional[Tensor] = None,
                                      n_rays: Optional[int] = None, prefix_trans: Optional[Tensor] = None
                                      ) -> Tuple[Tensor, Tensor]:
    """trans = exp(-exclusive_sum(sigma * dt)), alphas = 1 - exp(-sigma * dt) (packed samples)."""
    _, trans, alphas = render_weight_from_density(t_starts, t_ends, sigmas, packed_info, ray_indices, n_rays,
                                                  prefix_trans)
    return trans, alphas


def render_weight_from_density(t_starts: Tensor, t_ends: Tensor, sigmas: Tensor,
                               packed_info: Optional[Tensor] = None, ray_indices: Optional[Tensor] = None,
                               n_rays: Optional[int] = None, prefix_trans: Optional[Tensor] = None
                               ) -> Tuple[Tensor, Tensor, Tensor]:
    """(weights, trans, alphas) of packed samples (nerfacc.render_weight_from_density)."""
    assert t_starts.shape == t_ends.shape == sigmas.shape, "t_starts, t_ends and sigmas must match"
    if sigmas.dim() != 1:
        raise AcnError("the HIP render_weight_from_density takes packed (1-D) samples")
    starts, counts = _packed(packed_info, ray_indices, n_rays, sigmas.numel(), sigmas.device)
    w, tr, al = _PackedWeightsFn.apply(sigmas, t_starts.detach(), t_ends.detach(), starts, counts)
    if prefix_trans is not None:
        tr = tr * prefix_trans
        w = tr * al
    return w.to(sigmas.dtype), tr.to(sigmas.dtype), al.to(sigmas.dtype)


def render_visibility_from_density(t_starts: Tensor, t_ends: Tensor, sigmas: Tensor,
                                   packed_info: Optional[Tensor] = None, ray_indices: Optional[Tensor] = None,
                                   n_rays: Optional[int] = None, early_stop_eps: float = 1e-4,
                                   alpha_thre: float = 0.0, prefix_trans: Optional[Tensor] = None) -> Tensor:
    """Samples still visible: trans >= early_stop_eps (and alpha >= alpha_thre when > 0)."""
    with torch.no_grad():
        trans, alphas = render_transmittance_from_density(t_starts, t_ends, sigmas, packed_info, ray_indices,
                                                          n_rays, prefix_trans)
        vis = trans >= early_stop_eps
        if alpha_thre > 0.0:
            vis = vis & (alphas >= alpha_thre)
    return vis


class _PackedAccumulateFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, weights, values, ray_indices, starts, counts):
        out = occ_ops.packed_accumulate(weights, values, starts, counts)
        ctx.save_for_backward(weights, values if values is not None else None, ray_indices)
        ctx.has_values = values is not None
        return out

    @staticmethod
    def backward(ctx, g_out):
        weights, values, ray_indices = ctx.saved_tensors
        gw, gv = occ_ops.packed_accumulate_bwd(weights, values if ctx.has_values else None, ray_indices, g_out,
                                               ctx.needs_input_grad[0], ctx.has_values and ctx.needs_input_grad[1])
        return (None if gw is None else gw.view_as(weights), None if gv is None else gv.view_as(values),
                None, None, None)


def accumulate_along_rays(weights: Tensor, values: Optional[Tensor] = None, ray_indices: Optional[Tensor] = None,
                          n_rays: Optional[int] = None) -> Tensor:
    """(n_rays, C) per-ray sums of weights * values over ray-sorted packed samples."""
    assert weights.dim() == 1, "weights must be (M,)"
    if ray_indices is None or n_rays is None:
        raise AcnError("accumulate_along_rays needs ray_indices and n_rays for packed samples")
    pi = pack_info(ray_indices, n_rays)
    v = None if values is None else values.reshape(weights.shape[0], -1)
    out = _PackedAccumulateFn.apply(weights, v, ray_indices.long(), pi[:, 0].contiguous(), pi[:, 1].contiguous())
    return out.to(weights.dtype)


# ----------------------------------------------------------------------------------------------
def _enlarge_aabb(aabb: Tensor, factor: float) -> Tensor:
    center = (aabb[:3] + aabb[3:]) / 2
    extent = (aabb[3:] - aabb[:3]) / 2
    return torch.cat([center - extent * factor, center + extent * factor])


def _meshgrid3d(res: Tensor, device="cpu") -> Tensor:
    r = [int(v) for v in res.tolist()]
    g = torch.meshgrid([torch.arange(r[0], dtype=torch.long), torch.arange(r[1], dtype=torch.long),
                        torch.arange(r[2], dtype=torch.long)], indexing="ij")
    return torch.stack(g, dim=-1).to(device)


class OccGridEstimator(nn.Module):
    """Multi-level occupancy grid (nerfacc 0.5.3 OccGridEstimator), HIP-marched."""

    DIM: int = 3

    def __init__(self, roi_aabb, resolution=128, levels: int = 1, **kwargs) -> None:
        super().__init__()
        if "contraction_type" in kwargs:
            raise ValueError("`contraction_type` is not supported anymore by nerfacc >= 0.4")
        if isinstance(resolution, int):
            resolution = [resolution] * self.DIM
        if isinstance(resolution, (list, tuple)):
            resolution = torch.tensor(resolution, dtype=torch.int32)
        assert isinstance(resolution, Tensor) and resolution.shape[0] == self.DIM
        if isinstance(roi_aabb, (list, tuple)):
            roi_aabb = torch.tensor(roi_aabb, dtype=torch.float32)
        assert isinstance(roi_aabb, Tensor) and roi_aabb.shape[0] == self.DIM * 2
        self.cells_per_lvl = int(resolution.prod().item())
        self.levels = int(levels)
        self.register_buffer("resolution", resolution)
        self.register_buffer("aabbs", torch.zeros(levels, self.DIM * 2))
        self.register_buffer("occs", torch.zeros(self.levels * self.cells_per_lvl))
        self.register_buffer("binaries", torch.zeros([levels] + resolution.tolist(), dtype=torch.bool))
        self.aabbs = torch.stack([_enlarge_aabb(roi_aabb.detach().float().cpu(), 2 ** i) for i in range(levels)], 0) \
            .to(roi_aabb.device)
        self._bits = None
        self._bits_key = None
        self._host_key = None
        self._fixed_u = None

    # -------------------------------------------------------------------------- helpers
    @property
    def grid_indices(self) -> Tensor:
        return torch.arange(self.cells_per_lvl, device=self.occs.device)

    @property
    def grid_coords(self) -> Tensor:
        return _meshgrid3d(self.resolution.cpu(), self.occs.device).reshape(self.cells_per_lvl, self.DIM)

    def _host_meta(self):
        key = (self.aabbs.data_ptr(), self.aabbs._version, self.resolution.data_ptr(), self.resolution._version)
        if self._host_key != key:
            self._host_cache = ([list(map(float, r)) for r in self.aabbs.detach().cpu().tolist()],
                                [int(v) for v in self.resolution.cpu().tolist()])
            self._host_key = key
        return self._host_cache

    def occupancy_bits(self) -> Tensor:
        """1-bit-per-cell copy of `binaries` for the traversal kernel (rebuilt when it changes)."""
        b = self.binaries
        key = (b.data_ptr(), b._version, b.device)
        if self._bits is None or self._bits_key != key:
            self._bits = occ_ops.pack_bits(b)
            self._bits_key = key
        return self._bits

    # -------------------------------------------------------------------------- marching
    @torch.no_grad()
    def _sampling_packed(self, rays_o: Tensor, rays_d: Tensor, sigma_fn: Optional[Callable] = None,
                         alpha_fn: Optional[Callable] = None, near_plane: float = 0.0, far_plane: float = 1e10,
                         t_min: Optional[Tensor] = None, t_max: Optional[Tensor] = None,
                         render_step_size: float = 1e-3, early_stop_eps: float = 1e-4, alpha_thre: float = 0.0,
                         stratified: bool = False, cone_angle: float = 0.0, prefilter_aabb=None,
                         prefilter_near_far: Optional[Tensor] = None):
        """sampling() plus the packed layout: (ray_indices, t_starts, t_ends, chunk_starts, chunk_cnts)."""
        near_planes = torch.full_like(rays_o[..., 0], fill_value=near_plane)
        far_planes = torch.full_like(rays_o[..., 0], fill_value=far_plane)
        if t_min is not None:
            near_planes = torch.clamp(near_planes, min=t_min)
        if t_max is not None:
            far_planes = torch.clamp(far_planes, max=t_max)
        if stratified:  # `_fixed_u` (tests only) replays a recorded draw of the jitter uniforms
            u = self._fixed_u.to(near_planes) if self._fixed_u is not None else torch.rand_like(near_planes)
            near_planes += u * render_step_size
        aabbs, res = self._host_meta()
        ri, t0, t1, starts, counts = occ_ops.traverse(rays_o, rays_d, near_planes, far_planes, self.occupancy_bits(),
                                                      aabbs, res, render_step_size, cone_angle, prefilter_aabb,
                                                      prefilter_near_far)
        if (alpha_thre > 0.0 or early_stop_eps > 0.0) and (sigma_fn is not None or alpha_fn is not None):
            alpha_thre = min(alpha_thre, self.occs.mean().item())
            if sigma_fn is not None:
                sigmas = sigma_fn(t0, t1, ri) if t0.shape[0] != 0 else torch.empty((0,), device=t0.device)
                assert sigmas.shape == t0.shape, f"sigmas must have shape of (N,)! Got {sigmas.shape}"
                masks = render_visibility_from_density(t0, t1, sigmas, torch.stack([starts, counts], -1),
                                                       early_stop_eps=early_stop_eps, alpha_thre=alpha_thre)
            else:
                raise AcnError("alpha_fn marching is not used by the reference and not implemented")
            ri, t0, t1 = ri[masks], t0[masks], t1[masks]
            pi = pack_info(ri, rays_o.shape[0])
            starts, counts = pi[:, 0].contiguous(), pi[:, 1].contiguous()
        return ri, t0, t1, starts, counts

    @torch.no_grad()
    def sampling(self, rays_o: Tensor, rays_d: Tensor, sigma_fn: Optional[Callable] = None,
                 alpha_fn: Optional[Callable] = None, near_plane: float = 0.0, far_plane: float = 1e10,
                 t_min: Optional[Tensor] = None, t_max: Optional[Tensor] = None, render_step_size: float = 1e-3,
                 early_stop_eps: float = 1e-4, alpha_thre: float = 0.0, stratified: bool = False,
                 cone_angle: float = 0.0) -> Tuple[Tensor, Tensor, Tensor]:
        """(ray_indices, t_starts, t_ends) of the occupied samples along each ray."""
        ri, t0, t1, _, _ = self._sampling_packed(rays_o, rays_d, sigma_fn, alpha_fn, near_plane, far_plane, t_min,
                                                 t_max, render_step_size, early_stop_eps, alpha_thre, stratified,
                                                 cone_angle)
        return ri, t0, t1

    # -------------------------------------------------------------------------- grid maintenance
    @torch.no_grad()
    def mark_invisible_cells(self, K: Tensor, c2w: Tensor, width: int, height: int, near_plane: float = 0.0,
                             chunk: int = 32 ** 3) -> None:
        """occs <- -1 for cells no camera sees (in front of near_plane, inside the image)."""
        assert K.dim() == 3 and K.shape[1:] == (3, 3)
        assert c2w.dim() == 3 and (c2w.shape[1:] == (3, 4) or c2w.shape[1:] == (4, 4))
        assert K.shape[0] == c2w.shape[0] or K.shape[0] == 1 or c2w.shape[0] == 1
        aabbs, res = self._host_meta()
        Kd, Pd = K.to(self.occs.device), c2w.to(self.occs.device)
        for lvl, indices in enumerate(self._get_all_cells()):
            view = self.occs[lvl * self.cells_per_lvl:(lvl + 1) * self.cells_per_lvl]
            occ_ops.mark_invisible(Kd, Pd, width, height, near_plane, aabbs[lvl], res, indices, view)

    @torch.no_grad()
    def _get_all_cells(self) -> List[Tensor]:
        out = []
        gi = self.grid_indices
        for lvl in range(self.levels):
            cell_ids = lvl * self.cells_per_lvl + gi
            out.append(gi[self.occs[cell_ids] >= 0.0])
        return out

    @torch.no_grad()
    def _sample_uniform_and_occupied_cells(self, n: int) -> List[Tensor]:
        out = []
        for lvl in range(self.levels):
            uniform = torch.randint(self.cells_per_lvl, (n,), device=self.occs.device)
            cell_ids = lvl * self.cells_per_lvl + uniform
            uniform = uniform[self.occs[cell_ids] >= 0.0]
            occupied = torch.nonzero(self.binaries[lvl].flatten())[:, 0]
            if n < len(occupied):
                occupied = occupied[torch.randint(len(occupied), (n,), device=self.occs.device)]
            out.append(torch.cat([uniform, occupied], dim=0))
        return out

    @torch.no_grad()
    def _update(self, step: int, occ_eval_fn: Callable, occ_thre: float = 0.01, ema_decay: float = 0.95,
                warmup_steps: int = 256) -> None:
        if step < warmup_steps:
            lvl_indices = self._get_all_cells()
        else:
            lvl_indices = self._sample_uniform_and_occupied_cells(self.cells_per_lvl // 4)
        aabbs, res = self._host_meta()
        for lvl, indices in enumerate(lvl_indices):
            u = torch.rand(indices.shape[0], 3, device=self.occs.device, dtype=torch.float32)
            x = occ_ops.cell_points(indices, u, aabbs[lvl], res)
            occ = occ_eval_fn(x).squeeze(-1)
            occ_ops.ema(self.occs, lvl * self.cells_per_lvl + indices, occ, ema_decay)
        if not self.binaries.is_contiguous():
            self.binaries = self.binaries.contiguous()
        bits = self._bits if self._bits is not None and self._bits.device == self.occs.device else \
            torch.empty((self.occs.numel() + 31) // 32, device=self.occs.device, dtype=torch.int32)
        occ_ops.binarize(self.occs, occ_thre, self.binaries, bits)
        self._bits, self._bits_key = bits, (self.binaries.data_ptr(), self.binaries._version, self.binaries.device)

    @torch.no_grad()
    def update_every_n_steps(self, step: int, occ_eval_fn: Callable, occ_thre: float = 1e-2,
                             ema_decay: float = 0.95, warmup_steps: int = 256, n: int = 16) -> None:
        if not self.training:
            raise RuntimeError("You should only call this function only during training. Please call _update() "
                               "directly if you want to update the field during inference.")
        if step % n == 0 and self.training:
            self._update(step=step, occ_eval_fn=occ_eval_fn, occ_thre=occ_thre, ema_decay=ema_decay,
                         warmup_steps=warmup_steps)


# ----------------------------------------------------------------------------------------------
@torch.no_grad()
def ray_aabb_intersect(rays_o: Tensor, rays_d: Tensor, aabbs: Tensor, near_plane: float = -float("inf"),
                       far_plane: float = float("inf"), miss_value: float = float("inf")):
    """(t_mins, t_maxs, hits), each (n_rays, n_aabbs) (nerfacc.ray_aabb_intersect): the slab test the
    traversal kernel runs per level, exposed for callers that need it on its own (torch ops)."""
    o, d = rays_o[:, None, :], rays_d[:, None, :]
    lo, hi = aabbs[None, :, :3], aabbs[None, :, 3:]
    ta, tb = (lo - o) / d, (hi - o) / d
    tmin3, tmax3 = torch.minimum(ta, tb), torch.maximum(ta, tb)
    tmin = tmin3.amax(-1)
    tmax = tmax3.amin(-1)
    hits = tmax >= tmin
    t_mins = torch.where(hits, torch.clamp(tmin, min=near_plane), torch.full_like(tmin, miss_value))
    t_maxs = torch.where(hits, torch.clamp(tmax, max=far_plane), torch.full_like(tmax, miss_value))
    return t_mins, t_maxs, hits


@torch.no_grad()
def traverse_grids(rays_o: Tensor, rays_d: Tensor, binaries: Tensor, aabbs: Tensor, near_planes: Tensor,
                   far_planes: Tensor, step_size: float = 1e-3, cone_angle: float = 0.0):
    """Packed samples (ray_indices, t_starts, t_ends, chunk_starts, chunk_cnts) of traverse_grids."""
    res = list(binaries.shape[1:])
    aabb_list = [list(map(float, r)) for r in aabbs.detach().cpu().tolist()]
    return occ_ops.traverse(rays_o, rays_d, near_planes, far_planes, occ_ops.pack_bits(binaries), aabb_list, res,
                            step_size, cone_angle)
