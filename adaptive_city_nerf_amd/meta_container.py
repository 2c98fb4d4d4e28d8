"""K spatial experts with Voronoi routing and a background head
(reference interface: models/inr/meta_container.py:21-503).

Constructor, buffers (``scene_aabb_vec``, ``centroids``), submodule names (``submodules.{k}``,
``bg_dir_enc``, ``bg_mlp``) and methods match the reference.  ``forward`` without autograd is one
fused HIP launch (routing + every needed expert + soft blend in expert order);
``_routing`` and ``background_color`` run their own small HIP kernels; the autograd path
composes per-expert differentiable forwards exactly like the reference's index_select /
index_add_ loop, with routing weights from the HIP routing kernel.
"""
from __future__ import annotations

from typing import Dict, List, Literal, Optional, OrderedDict, Tuple

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import ops
from .encodings import FrequencyEncoder, SHEncoder
from .meta_ngp import MetaNGP
from .metamodule import MetaModule


def build_expert(nerf_variant: str, **nerf_kwargs) -> nn.Module:
    """Factory for one expert (meta_container.py:14-18)."""
    if nerf_variant == "instant":
        return MetaNGP(**nerf_kwargs)
    raise NotImplementedError("only the Instant-NGP expert ('instant') is on the MI355X hot path "
                              "(the reference's MetaNeRF variant is itself broken, SURVEY §2)")


class _BackgroundFn(torch.autograd.Function):
    """The SH-4 background head with the HIP forward (acn_background_fwd) and backward
    (acn_background_bwd: the 643 parameter gradients in two launches instead of the ~15 of the torch
    chain's autograd graph).  First-order: the directions get no gradient."""

    @staticmethod
    def forward(ctx, d, bg, w1, b1, w2, b2):
        ctx.save_for_backward(d)
        ctx.bg = bg
        ctx.shapes = [t.shape for t in (w1, b1, w2, b2)]
        return ops.background_fwd(d, bg)

    @staticmethod
    def backward(ctx, g):
        (d,) = ctx.saved_tensors
        grads = [torch.empty(sh, device=d.device, dtype=torch.float32) for sh in ctx.shapes]
        ops.background_bwd(d, ctx.bg, g.contiguous(), grads)
        return (None, None, *[gr if need else None for gr, need in zip(grads, ctx.needs_input_grad[2:])])


class MetaContainer(MetaModule):
    def __init__(self, num_submodules: int, centroids: torch.Tensor, aabb: torch.Tensor,
                 nerf_variant: Literal["instant", "vanilla"] = "instant", boundary_margin: float = 1.0,
                 cluster_2d: bool = True, joint_training: bool = False, use_bg_nerf: bool = True, bg_hidden: int = 32,
                 bg_encoding: Literal["spherical", "fourier"] = "spherical", occ_conf: Optional[Dict] = None,
                 **nerf_kwargs):
        super().__init__()
        assert num_submodules > 0
        assert centroids.ndim == 2 and centroids.size(0) == num_submodules
        assert boundary_margin >= 1.0
        if num_submodules > ops._lib.ACN_MAX_EXPERTS:
            raise ValueError(f"at most {ops._lib.ACN_MAX_EXPERTS} experts are supported")
        occ_conf = occ_conf or {}
        self.register_buffer("scene_aabb_vec", torch.cat([aabb[0], aabb[1]], dim=0).float(), persistent=True)
        self.register_buffer("centroids", centroids.to(torch.float32), persistent=True)
        self.use_occ = bool(occ_conf.get("use_occ", False))
        self.boundary_margin = float(boundary_margin)
        self.cluster_2d = bool(cluster_2d)
        self.joint_training = bool(joint_training)
        self._coord_idx = (1, 2) if self.cluster_2d else (0, 1, 2)
        self.nerf_variant = nerf_variant
        self.dim_out = 4
        expert_box_list = nerf_kwargs.pop("expert_box_list")
        base = {**nerf_kwargs, "occ_conf": occ_conf}
        self.submodules = nn.ModuleList()
        for box in expert_box_list:
            self.submodules.append(build_expert(nerf_variant, **{**base, "scene_box": box}))
        self.use_bg_nerf = bool(use_bg_nerf)
        if self.use_bg_nerf:
            if bg_encoding == "spherical":
                self.bg_dir_enc = SHEncoder(levels=4, implementation="tcnn")
            else:
                self.bg_dir_enc = FrequencyEncoder(pe_dim=4, include_input=True, use_pi=False)  # as reference
            in_ch = self.bg_dir_enc.out_dim
            self.bg_hidden_dim = int(bg_hidden)
            self.bg_mlp = nn.Sequential(nn.Linear(in_ch, self.bg_hidden_dim, bias=True), nn.ReLU(),
                                        nn.Linear(self.bg_hidden_dim, 3, bias=True), nn.Sigmoid())

    # ---------------------------------------------------------------- kernel-side descriptions
    def routing_spec(self):
        c = self.centroids
        key = (c.data_ptr(), c._version, self.boundary_margin, self.cluster_2d)
        if getattr(self, "_routing_key", None) != key:
            self._routing_cache = ops.make_routing(c, len(self.submodules), self.cluster_2d, self.boundary_margin)
            self._routing_key = key
        return self._routing_cache

    def expert_specs(self, params=None) -> List[ops.ExpertSpec]:
        K = len(self.submodules)
        sub = [self.get_subdict(params, f"submodules.{k}") for k in range(K)] if params is not None else [None] * K
        return [self.submodules[k].expert_spec(sub[k]) for k in range(K)]

    def packed_weights(self, specs, routing, active_module=None, params=None):
        """Packed MFMA weight image for the fused kernels, cached while no owned weight changed."""
        if params is not None:
            return ops.pack_experts(specs, routing, active_module)
        subs = self.submodules if active_module is None else [self.submodules[active_module]]
        key = (active_module,) + tuple((id(t), t.data_ptr(), t._version) for s in subs
                                      for t in s._mlp_tensors(None).values())
        if not hasattr(self, "_pack_cache"):
            self._pack_cache = ops.PackCache()
        return self._pack_cache.get(specs, routing, active_module, key)

    def background_spec(self):
        if not self.use_bg_nerf:
            raise RuntimeError("background_color called but use_bg_nerf=False")
        if not isinstance(self.bg_dir_enc, SHEncoder) or self.bg_dir_enc.levels != 4:
            raise ops.AcnError("the HIP background head implements the spherical (SH-4) encoding")
        m = self.bg_mlp
        return ops.make_background("mlp", mlp={"0.weight": m[0].weight, "0.bias": m[0].bias,
                                               "2.weight": m[2].weight, "2.bias": m[2].bias})

    def uses_grad(self, params=None) -> bool:
        K = len(self.submodules)
        sub = [self.get_subdict(params, f"submodules.{k}") for k in range(K)] if params is not None else [None] * K
        return any(self.submodules[k].uses_grad(sub[k]) for k in range(K))

    # ---------------------------------------------------------------- routing
    def _routing(self, pts: torch.Tensor) -> Tuple[Optional[torch.Tensor], Optional[torch.Tensor]]:
        """Soft weights (N,K) when boundary_margin > 1, else hard assignment (N,) (:97-134)."""
        assert pts.dim() == 2 and pts.shape[-1] == 3, "pts must be (N,3)"
        assert self.centroids.shape[0] > 0, "No centroids provided."
        with torch.no_grad():
            return ops.routing_fwd(pts.to(self.centroids.device), self.routing_spec())

    def _sub_params(self, params):
        K = len(self.submodules)
        return [self.get_subdict(params, f"submodules.{k}") for k in range(K)] if params is not None else [None] * K

    # ---------------------------------------------------------------- network calls
    def color(self, xyz: torch.Tensor, dirs: torch.Tensor, params: Optional[OrderedDict] = None,
              active_module: Optional[int] = None) -> torch.Tensor:
        assert xyz.dim() == 2 and xyz.shape[-1] == 3, "xyz must be (N,3)"
        assert dirs.dim() == 2 and dirs.shape[-1] == 3, "dirs must be (N,3)"
        dirs = F.normalize(dirs.to(xyz.device), dim=-1)
        sub_params = self._sub_params(params)
        if active_module is not None:
            sub = self.submodules[active_module]
            dens = sub.density(xyz, params=sub_params[active_module], return_feats=True)
            return sub.color(dirs, dens["geo_feat"], params=sub_params[active_module])
        weights, hard = self._routing(xyz)
        results = xyz.new_zeros(xyz.shape[0], 3)
        for k, sub in enumerate(self.submodules):
            sel = ((weights[:, k] > 0) if weights is not None else (hard == k)).nonzero(as_tuple=False).squeeze(1)
            if sel.numel() == 0:
                continue
            dens = sub.density(xyz.index_select(0, sel), params=sub_params[k], return_feats=True)
            rgb = sub.color(dirs.index_select(0, sel), dens["geo_feat"], params=sub_params[k])
            if weights is not None:
                results.index_add_(0, sel, rgb * weights[:, k].index_select(0, sel).unsqueeze(1))
            else:
                results.index_copy_(0, sel, rgb)
        return results

    def density(self, xyz: torch.Tensor, params: Optional[OrderedDict] = None,
                active_module: Optional[int] = None) -> torch.Tensor:
        assert xyz.dim() == 2 and xyz.shape[-1] == 3, "xyz must be (N,3)"
        sub_params = self._sub_params(params)
        if active_module is not None:
            return self.submodules[active_module].density(xyz, params=sub_params[active_module]).squeeze(-1)
        weights, hard = self._routing(xyz)
        sig = xyz.new_zeros(xyz.shape[0])
        for k, sub in enumerate(self.submodules):
            sel = ((weights[:, k] > 0) if weights is not None else (hard == k)).nonzero(as_tuple=False).squeeze(1)
            if sel.numel() == 0:
                continue
            s = sub.density(xyz.index_select(0, sel), params=sub_params[k]).to(xyz.dtype).squeeze(-1)
            if weights is not None:
                sig.index_add_(0, sel, s * weights[:, k].index_select(0, sel))
            else:
                sig.index_copy_(0, sel, s)
        return sig

    def forward(self, x: torch.Tensor, params: Optional[OrderedDict] = None,
                active_module: Optional[int] = None) -> torch.Tensor:
        """Routed forward (:275-343): x (N, D>=6) -> (N, 4) [rgb, sigma]."""
        assert x.dim() == 2 and x.shape[-1] >= 6, "x must be (N,D>=6)"
        # the reference's experts assert exactly 6 columns (meta_ngp.py:236)
        assert x.shape[-1] == 6, f"Expected (...,6) [xyz,dir], got {x.shape}"
        sub_params = self._sub_params(params)
        if active_module is not None:
            return self.submodules[active_module](x, params=sub_params[active_module])
        if not self.uses_grad(params) and all(s._fusable for s in self.submodules):
            specs, routing = self.expert_specs(params), self.routing_spec()
            return ops.field_fwd(x, specs, routing, packed=self.packed_weights(specs, routing, None, params))
        weights, hard = self._routing(x[:, :3])
        results = x.new_zeros(x.shape[0], self.dim_out)
        for k, sub in enumerate(self.submodules):
            sel = ((weights[:, k] > 0) if weights is not None else (hard == k)).nonzero(as_tuple=False).squeeze(1)
            if sel.numel() == 0:
                continue
            yk = sub(x.index_select(0, sel), params=sub_params[k])
            if weights is not None:
                results = results.index_add(0, sel, yk * weights[:, k].index_select(0, sel).unsqueeze(1))
            else:
                results = results.index_copy(0, sel, yk)
        return results

    # ---------------------------------------------------------------- background
    def background_color(self, d: torch.Tensor) -> torch.Tensor:
        """SH(4) -> Linear -> ReLU -> Linear -> Sigmoid of the ray direction (:347-382)."""
        if not self.use_bg_nerf:
            raise RuntimeError("background_color called but use_bg_nerf=False")
        if d.dim() not in (2, 3):
            raise ValueError(f"background_color expects (N,3) or (B,N,3), got {tuple(d.shape)}")
        shape = d.shape
        if torch.is_grad_enabled() and any(p.requires_grad for p in self.bg_mlp.parameters()):
            from .ray_rendering import _second_order
            if d.is_cuda and not d.requires_grad and not _second_order():
                try:
                    bg, keep = self.background_spec()
                except ops.AcnError:
                    bg = None
                if bg is not None:   # fused HIP forward + backward (acn_background_fwd / _bwd)
                    m = self.bg_mlp
                    return _BackgroundFn.apply(d.reshape(-1, 3).float().contiguous(), bg, m[0].weight, m[0].bias,
                                               m[2].weight, m[2].bias).view(*shape[:-1], 3)
            dn = F.normalize(d.reshape(-1, 3), dim=-1)
            enc = self.bg_dir_enc(dn).to(self.bg_mlp[0].weight.dtype)
            return self.bg_mlp(enc).view(*shape[:-1], 3)
        bg, keep = self.background_spec()
        return ops.background_fwd(d.reshape(-1, 3), bg).view(*shape[:-1], 3)

    # ---------------------------------------------------------------- occupancy (meta_container.py:386-462)
    def maybe_update_expert_occupancies(self, step: int, params=None) -> None:
        for sub in self.submodules:
            sub.maybe_update_occ_grid(step, params)

    def freeze_expert_occupancies(self, flag: bool) -> None:
        for sub in self.submodules:
            sub.occ_frozen = flag

    @torch.no_grad()
    def premark_invisible_expert_cells(self, metas, near_plane: float = 0.0, chunk: int = 32 ** 3) -> List[int]:
        """One-time visibility pruning of every expert's grid; returns the cells marked per expert."""
        if self.cells_premarked or not self.use_occ:
            return [0] * len(self.submodules)
        marked = []
        for k, expert in enumerate(self.submodules):
            expert.premark_invisible_cells(metas, near_plane=float(near_plane), chunk=chunk)
            n_marked = int((expert.occ_grid.occs < 0).sum().item()) if hasattr(expert.occ_grid, "occs") else 0
            total = expert.occ_grid.occs.numel() if hasattr(expert.occ_grid, "occs") else 0
            marked.append(n_marked)
            print(f"[OCC] container: expert#{k} cams={len(metas)} marked_invisible={n_marked} / {total} "
                  f"({100.0 * n_marked / max(1, total):.2f}%)")
        print("[OCC] container: premark complete for all experts.")
        return marked

    @property
    def occ_ready(self) -> bool:
        return all(sub.occ_ready for sub in self.submodules)

    @property
    def cells_premarked(self) -> bool:
        return all(sub.occ_premarked for sub in self.submodules)

    def get_param_groups(self) -> Dict[str, Dict]:
        enc, sig, col, bg = [], [], [], []
        for sub in self.submodules:
            g = sub.get_param_groups()
            enc += list(g["encoding"]["params"])
            sig += list(g["sigma"]["params"])
            col += list(g["color"]["params"])
        if self.use_bg_nerf:
            bg += list(self.bg_dir_enc.parameters()) + list(self.bg_mlp.parameters())
        groups = {}
        if enc:
            groups["encoding"] = {"params": enc}
        if sig:
            groups["sigma"] = {"params": sig}
        if col:
            groups["color"] = {"params": col}
        if bg:
            groups["background"] = {"params": bg}
        return groups
