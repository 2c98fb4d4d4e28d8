"""One Instant-NGP expert (reference interface: models/inr/meta_ngp.py:15-241).

Same constructor, submodule names (state-dict keys such as ``xyz_encoder.hash_table``,
``sigma_trunk.0.linear.weight``, ``color_mlp.2.bias``), buffers and methods as the reference.
``forward`` without autograd runs the fused HIP field kernel (hash grid -> sigma trunk -> heads ->
SH -> colour MLP in one launch, fp32 MFMA); with autograd it composes the HIP hash-grid
forward/backward with the fast-weight MetaLinear chain so gradients reach the table and every
(fast) weight.  The occupancy-grid path (use_occ, nerfacc) is outside this round's scope.
"""
from __future__ import annotations

from typing import Dict, Literal, Optional, Union

import torch
from torch import Tensor

from . import ops
from .encodings import FrequencyEncoder, HashGridEncoder, SHEncoder
from .metamodule import MetaLayerBlock, MetaLinear, MetaModule, MetaSequential
from .scene_box import SceneBox
from .trunc_exp import trunc_exp


def _needs_grad(*ts) -> bool:
    return torch.is_grad_enabled() and any(t is not None and t.requires_grad for t in ts)


class MetaNGP(MetaModule):
    def __init__(self, *, occ_conf: Dict, scene_box: SceneBox, hidden: int = 64, sigma_depth: int = 2,
                 color_hidden: int = 64, geo_feat_dim: int = 15, color_depth: int = 3, use_sigmoid_rgb: bool = True,
                 hash_enc_conf=None, dir_encoding: Literal["spherical", "frequency"] = "spherical", **kwargs) -> None:
        super().__init__()
        self.register_buffer("aabb_extent", scene_box.extent)
        self.register_buffer("enc_eps", torch.tensor(1e-6, dtype=torch.float32), persistent=False)
        hash_enc_conf = hash_enc_conf or {}
        occ_conf = occ_conf or {}
        self.use_occ = bool(occ_conf.get("use_occ", False))
        if self.use_occ:
            raise NotImplementedError("occupancy-grid rendering (nerfacc) is not part of this build yet "
                                      "(SURVEY §8(f) rank 1); construct with occ_conf={'use_occ': False}")
        self.geo_feat_dim = int(geo_feat_dim)
        self.use_sigmoid_rgb = bool(use_sigmoid_rgb)
        self.scene_box = scene_box
        aabb = scene_box.aabb
        assert isinstance(aabb, torch.Tensor) and aabb.shape == (2, 3)
        self.xyz_encoder = HashGridEncoder(
            levels=hash_enc_conf.get("levels", 4), min_res=hash_enc_conf.get("min_res", 16),
            max_res=hash_enc_conf.get("max_res", 4096), log2_hashmap_size=hash_enc_conf.get("log2_hashmap_size", 19),
            features_per_level=hash_enc_conf.get("features_per_level", 2),
            interpolation=hash_enc_conf.get("interpolation", "Linear"))
        in_ch_xyz = self.xyz_encoder.out_dim
        dir_encoding = dir_encoding.lower()
        if dir_encoding == "frequency":
            self.dir_encoder = FrequencyEncoder(in_dim=3, pe_dim=4, include_input=True, use_pi=False)
        elif dir_encoding == "spherical":
            self.dir_encoder = SHEncoder(levels=4)
        else:
            raise ValueError(f"Unsupported dir_encoding: {dir_encoding}")
        in_ch_dir = self.dir_encoder.out_dim
        trunk, last = [], in_ch_xyz
        for _ in range(max(int(sigma_depth), 0)):
            trunk.append(MetaLayerBlock(last, hidden, activation="relu"))
            last = hidden
        self.sigma_trunk = MetaSequential(*trunk)
        self.sigma_head = MetaLinear(last, 1)
        with torch.no_grad():
            self.sigma_head.bias.fill_(-1.0)
        self.geo_head = MetaLinear(last, self.geo_feat_dim)
        self.sigma_act = trunc_exp
        cmlp, last = [], self.geo_feat_dim + in_ch_dir
        for _ in range(max(int(color_depth), 0)):
            cmlp.append(MetaLayerBlock(last, color_hidden, activation="relu"))
            last = color_hidden
        cmlp.append(MetaLinear(last, 3))
        self.color_mlp = MetaSequential(*cmlp)
        self.rgb_act = torch.nn.Sigmoid() if self.use_sigmoid_rgb else torch.nn.Identity()
        self.occ_ready = False
        self.occ_premarked = False
        self.occ_frozen = False
        self._fusable = (isinstance(self.dir_encoder, SHEncoder) and self.xyz_encoder.levels == 16
                         and self.xyz_encoder.features_per_level == 2 and int(sigma_depth) == 2 and hidden == 64
                         and self.geo_feat_dim == 15 and int(color_depth) == 2 and color_hidden == 64
                         and self.use_sigmoid_rgb)

    # ------------------------------------------------------------------ encoding helpers
    def _world_to_unit(self, x: Tensor) -> Tensor:
        x01 = (x - self.scene_box.min.to(x.device)) / self.aabb_extent
        return x01.clamp(self.enc_eps, 1.0 - self.enc_eps)

    def _enc_xyz(self, x_world: Tensor) -> Tensor:
        return self.xyz_encoder(self._world_to_unit(x_world))

    def _enc_dir(self, d: Tensor) -> Tensor:
        d = d / d.norm(dim=-1, keepdim=True).clamp_min_(1e-9)
        return self.dir_encoder(d)

    # ------------------------------------------------------------------ fused-path plumbing
    def _mlp_tensors(self, params: Optional[Dict[str, Tensor]]) -> Dict[str, Tensor]:
        own = dict(self.meta_named_parameters())
        if params is None:
            return own
        return {k: params.get(k, v) for k, v in own.items()}

    def _host_box(self):
        """(min, extent) as host floats, cached on the tensors' identity and version counters so
        a render call never synchronises with the device (load_state_dict bumps the version)."""
        mn, ext = self.scene_box.min, self.aabb_extent
        key = (mn.data_ptr(), mn._version, ext.data_ptr(), ext._version)
        if getattr(self, "_box_key", None) != key:
            self._box_cache = (mn.detach().float().cpu().tolist(), ext.detach().float().cpu().tolist())
            self._box_key = key
        return self._box_cache

    def expert_spec(self, params: Optional[Dict[str, Tensor]] = None) -> ops.ExpertSpec:
        """Device description of this expert for the fused kernels (fast weights from params)."""
        if not self._fusable:
            raise ops.AcnError("the fused HIP field implements the reference configuration (L=16, F=2, sigma 2x64, "
                               "geo 15, SH-4, colour 2x64, sigmoid rgb; nerf_runner.py:102-121)")
        enc = self.xyz_encoder
        mn, ext = self._host_box()
        return ops.ExpertSpec(enc.hash_table, enc._res_host, enc.log2_hashmap_size, enc._interp_code, mn, ext,
                              self._mlp_tensors(params))

    def packed_weights(self, spec, routing, params=None):
        if params is not None:
            return ops.pack_experts([spec], routing, 0)
        key = tuple((id(t), t.data_ptr(), t._version) for t in self.meta_parameters())
        if not hasattr(self, "_pack_cache"):
            self._pack_cache = ops.PackCache()
        return self._pack_cache.get([spec], routing, 0, key)

    def uses_grad(self, params: Optional[Dict[str, Tensor]] = None) -> bool:
        tensors = [self.xyz_encoder.hash_table] + list(self._mlp_tensors(params).values())
        return _needs_grad(*tensors)

    # ------------------------------------------------------------------ network calls
    def color(self, d: Tensor, geo_feat: Tensor, params: Optional[Dict[str, Tensor]] = None) -> Tensor:
        d_enc = self._enc_dir(d)
        h = torch.cat([geo_feat, d_enc.to(geo_feat.dtype)], dim=-1)
        h = self.color_mlp(h, params=self.get_subdict(params, "color_mlp"))
        return self.rgb_act(h)

    def density(self, x: Tensor, params: Optional[Dict[str, Tensor]] = None,
                return_feats: bool = False) -> Union[Tensor, Dict[str, Tensor]]:
        h = self._enc_xyz(x)
        h = self.sigma_trunk(h, params=self.get_subdict(params, "sigma_trunk"))
        sigma = self.sigma_act(self.sigma_head(h, params=self.get_subdict(params, "sigma_head")))
        if not return_feats:
            return sigma
        geo = self.geo_head(h, params=self.get_subdict(params, "geo_head"))
        return {"sigma": sigma, "geo_feat": geo}

    def forward(self, x_d: Tensor, params=None) -> Tensor:
        """[xyz(3), dir(3)] -> [rgb(3), sigma(1)] (meta_ngp.py:226-241)."""
        assert x_d.shape[-1] == 6, f"Expected (...,6) [xyz,dir], got {x_d.shape}"
        if self._fusable and not self.uses_grad(params):
            from ._lib import acn_routing
            r = acn_routing()
            r.K, r.cluster_2d, r.boundary_margin = 1, 1, 1.0
            flat = x_d.reshape(-1, 6)
            spec = self.expert_spec(params)
            return ops.field_fwd(flat, [spec], r, active_module=0,
                                 packed=self.packed_weights(spec, r, params)).view(*x_d.shape[:-1], 4)
        x, d = x_d[..., :3], x_d[..., 3:6]
        dens = self.density(x, params=params, return_feats=True)
        rgb = self.color(d, dens["geo_feat"], params=params)
        return torch.cat([rgb, dens["sigma"]], dim=-1)

    # ------------------------------------------------------------------ occupancy (out of scope)
    def maybe_update_occ_grid(self, step: int, params: Optional[Dict[str, Tensor]] = None) -> None:
        return None  # use_occ is always False in this build (reference early-returns the same way)

    def premark_invisible_cells(self, *a, **k) -> None:
        return None

    def occupancy_marching(self, *a, **k):
        raise NotImplementedError("occupancy marching (nerfacc) is not part of this build (SURVEY §8(f))")

    def get_param_groups(self) -> Dict[str, Dict]:
        return {
            "encoding": {"params": list(self.xyz_encoder.parameters())},
            "sigma": {"params": list(self.sigma_trunk.parameters()) + list(self.sigma_head.parameters())
                      + list(self.geo_head.parameters())},
            "color": {"params": list(self.color_mlp.parameters())},
        }
