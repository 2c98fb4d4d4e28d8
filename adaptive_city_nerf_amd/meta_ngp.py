"""One Instant-NGP expert (reference interface: models/inr/meta_ngp.py:15-241).

Same constructor, submodule names (state-dict keys such as ``xyz_encoder.hash_table``,
``sigma_trunk.0.linear.weight``, ``color_mlp.2.bias``), buffers and methods as the reference.
``forward`` without autograd runs the fused HIP field kernel (hash grid -> sigma trunk -> heads ->
SH -> colour MLP in one launch, fp32 MFMA); with autograd it composes the HIP hash-grid
forward/backward with the fast-weight MetaLinear chain so gradients reach the table and every
(fast) weight.  With ``occ_conf['use_occ']`` the expert owns an occupancy grid (the nerfacc
OccGridEstimator surface of .nerfacc, HIP-marched) with the reference's premark / update /
marching methods (meta_ngp.py:242-443).
"""
from __future__ import annotations

import math
from typing import Dict, List, Literal, Optional, Tuple, Union

import torch
from torch import Tensor

from . import ops
from .encodings import FrequencyEncoder, HashGridEncoder, SHEncoder
from .nerfacc import OccGridEstimator
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
        if self.use_occ:  # meta_ngp.py:100-141
            rss = occ_conf.get("render_step_size")
            self.render_step_size = float(rss) if rss is not None else float(scene_box.get_diagonal_length()) / 1000.0
            self.occ_thre: float = float(occ_conf.get("occ_thre", 1e-2))
            self.alpha_thre: float = float(occ_conf.get("alpha_thre", 1e-2))
            self.cone_angle: float = float(occ_conf.get("cone_angle", 1.0 / 256.0))
            self.near_plane: float = float(occ_conf.get("near_plane", 0.05))
            self.far_plane: float = float(occ_conf.get("far_plane", 1e3))
            self.occ_update_interval: int = int(occ_conf.get("update_interval", 16))
            self.occ_warmup_steps: int = int(occ_conf.get("warmup_steps", 256))
            self.occ_cosine_anneal = bool(occ_conf.get("cosine_anneal", True))
            self.occ_alpha_thre_start: float = float(occ_conf.get("alpha_thre_start", 0.0))
            self.occ_alpha_thre_end: float = float(occ_conf.get("alpha_thre_end", self.alpha_thre))
            self.occ_ema_decay: float = float(occ_conf.get("ema_decay", 0.95))
            self.occ_resolution: int = int(occ_conf.get("resolution", 128))
            self.occ_levels: int = int(occ_conf.get("levels", 4))
            scene_aabb = torch.cat([self.scene_box.min, self.scene_box.max]).flatten()
            self.register_buffer("scene_aabb", scene_aabb)
            self.occ_grid = OccGridEstimator(roi_aabb=self.scene_aabb, resolution=self.occ_resolution,
                                             levels=self.occ_levels)
            self._check_aabb()
            self.occ_frozen = bool(occ_conf.get("occ_frozen", False))
            self.occ_ready = bool(occ_conf.get("occ_ready", False))
            self.num_occ_updates = 0
            self.occ_premarked = False
        self._fusable = (isinstance(self.dir_encoder, SHEncoder) and self.xyz_encoder.levels == 16
                         and self.xyz_encoder.features_per_level == 2 and int(sigma_depth) == 2 and hidden == 64
                         and self.geo_feat_dim == 15 and int(color_depth) == 2 and color_hidden == 64
                         and self.use_sigmoid_rgb)

    # ------------------------------------------------------------------ encoding helpers
    def _check_aabb(self) -> None:
        aabb = self.scene_aabb
        assert aabb.dtype == torch.float32 and aabb.isfinite().all()
        assert aabb.numel() == 6
        mn, mx = aabb[:3], aabb[3:]
        if not (mn < mx).all():
            raise ValueError(f"AABB invalid: min>=max ({mn} vs {mx})")
        assert aabb.device == self.occ_grid.aabbs.device

    def _box_min_on(self, device) -> Tensor:
        """scene_box.min on ``device``, cached on the tensor's identity / version (no per-call host copy,
        so the training step stays capturable in a HIP graph)."""
        mn = self.scene_box.min
        if mn.device == device:
            return mn
        key = (mn.data_ptr(), mn._version, str(device))
        if getattr(self, "_min_dev_key", None) != key:
            self._min_dev = mn.to(device)
            self._min_dev_key = key
        return self._min_dev

    def _world_to_unit(self, x: Tensor) -> Tensor:
        x01 = (x - self._box_min_on(x.device)) / self.aabb_extent
        return x01.clamp(self.enc_eps, 1.0 - self.enc_eps)

    def _enc_xyz(self, x_world: Tensor) -> Tensor:
        return self.xyz_encoder(self._world_to_unit(x_world))

    def _enc_dir(self, d: Tensor) -> Tensor:
        d = d / d.norm(dim=-1, keepdim=True).clamp_min_(1e-9)
        return self.dir_encoder(d)

    # ------------------------------------------------------------------ fused-path plumbing
    def _meta_slots(self):
        """(name, owning module's _parameters dict, key) of every meta parameter, in meta_named_parameters
        order, found once: a render call reads the current tensors through these slots instead of walking
        the module tree (the walk was most of the ~0.3 ms of host time per render_rays call)."""
        slots = self.__dict__.get("_meta_slot_cache")
        if slots is None:
            slots = []
            for name, _ in self.meta_named_parameters():
                path, _, pname = name.rpartition(".")
                mod = self.get_submodule(path) if path else self
                slots.append((name, mod._parameters, pname))
            self.__dict__["_meta_slot_cache"] = slots
        return slots

    def _mlp_tensors(self, params: Optional[Dict[str, Tensor]]) -> Dict[str, Tensor]:
        own = {n: d[k] for n, d, k in self._meta_slots()}
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
        mlp = self._mlp_tensors(params)
        if params is not None or not all(t.dtype == torch.float32 and t.is_contiguous()
                                         for t in [enc.hash_table, *mlp.values()]):   # copies: never cached
            return ops.ExpertSpec(enc.hash_table, enc._res_host, enc.log2_hashmap_size, enc._interp_code, mn, ext, mlp)
        # module weights: the spec holds pointers only, so it is reused while every tensor keeps its storage
        key = (self._box_key, enc.hash_table.data_ptr(), enc.log2_hashmap_size, enc._interp_code,
               tuple(enc._res_host)) + tuple((id(t), t.data_ptr()) for t in mlp.values())
        cache = self.__dict__.get("_spec_cache")
        if cache is None or cache[0] != key:
            cache = (key, ops.ExpertSpec(enc.hash_table, enc._res_host, enc.log2_hashmap_size, enc._interp_code, mn,
                                         ext, mlp))
            self.__dict__["_spec_cache"] = cache
        return cache[1]

    def packed_weights(self, spec, routing, params=None):
        if params is not None:
            return ops.pack_experts([spec], routing, 0)
        key = tuple((id(t), t.data_ptr(), t._version) for t in self._mlp_tensors(None).values())
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
        if not return_feats and x.is_cuda and self._fusable and not self.uses_grad(params):
            # no autograd (occupancy updates / marching visibility): the fused field kernel; the
            # direction input only feeds the colour branch, whose output is dropped
            flat = x.reshape(-1, 3)
            sig = self.forward(torch.cat([flat, torch.zeros_like(flat)], dim=-1), params=params)[:, 3:4]
            return sig.reshape(*x.shape[:-1], 1)
        h = self._enc_xyz(x)
        h = self.sigma_trunk(h, params=self.get_subdict(params, "sigma_trunk"))
        sigma = self.sigma_act(self.sigma_head(h, params=self.get_subdict(params, "sigma_head")))
        if not return_feats:
            return sigma
        geo = self.geo_head(h, params=self.get_subdict(params, "geo_head"))
        return {"sigma": sigma, "geo_feat": geo}

    def _fused_train_ok(self, x: Tensor) -> bool:
        from .ray_rendering import _second_order
        return x.is_cuda and self._fusable and x.dtype == torch.float32 and not _second_order()

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
        if self._fused_train_ok(x_d):
            # training: hash grid (HIP, autograd to the table) + the whole MLP fwd/bwd on MFMA
            flat = x_d.reshape(-1, 6)
            h0 = self._enc_xyz(flat[:, :3])
            with torch.no_grad():
                sh = self._enc_dir(flat[:, 3:6])
            ws = [t.contiguous() for t in self._mlp_tensors(params).values()]
            out = _FusedMLPFn.apply(h0.contiguous(), sh.contiguous(), *ws)
            return out.view(*x_d.shape[:-1], 4)
        dens = self.density(x, params=params, return_feats=True)
        rgb = self.color(d, dens["geo_feat"], params=params)
        return torch.cat([rgb, dens["sigma"]], dim=-1)

    # ------------------------------------------------------------------ occupancy (meta_ngp.py:242-443)
    def _anneal_alpha_thre(self, step: int) -> None:
        """Ramp alpha threshold from start to end over warmup, then hold."""
        if step < self.occ_warmup_steps:
            t = step / max(1, self.occ_warmup_steps - 1)
            if self.occ_cosine_anneal:
                cos = 0.5 * (1 - math.cos(math.pi * t))
                self.alpha_thre = (1 - cos) * self.occ_alpha_thre_start + cos * self.occ_alpha_thre_end
            else:
                self.alpha_thre = (1 - t) * self.occ_alpha_thre_start + t * self.occ_alpha_thre_end
        else:
            self.alpha_thre = self.occ_alpha_thre_end

    @torch.no_grad()
    def _build_intrinsics_from_metadata(self, mds: List, device: torch.device) -> Tensor:
        """(N,3,3) K matrices from metadata intrinsics (9 values, or [fx, fy, cx, cy])."""
        def _make_K(md) -> Tensor:
            Kraw = torch.as_tensor(md.intrinsics, dtype=torch.float32)
            if Kraw.numel() == 9:
                return Kraw.view(3, 3)
            if Kraw.numel() == 4:
                fx, fy, cx, cy = Kraw.unbind()
                return torch.tensor([[fx, 0.0, cx], [0.0, fy, cy], [0.0, 0.0, 1.0]], dtype=torch.float32)
            raise ValueError(f"Unsupported intrinsics shape: {tuple(Kraw.shape)}")
        return torch.stack([_make_K(md) for md in mds], dim=0).to(device=device, dtype=torch.float32)

    @torch.no_grad()
    def _build_c2w_rdf_from_metadata(self, mds: List, device: torch.device) -> Tensor:
        """c2w (N,3,4) or (N,4,4) with the rotation converted from RUB to RDF."""
        c2w = torch.stack([torch.as_tensor(md.c2w, dtype=torch.float32) for md in mds], dim=0)
        C3 = torch.diag(torch.tensor([1.0, -1.0, -1.0], dtype=torch.float32))
        if c2w.shape[1:] == (3, 4):
            R_rdf = torch.einsum("nij,jk->nik", c2w[:, :3, :3], C3)
            c2w_rdf = torch.cat([R_rdf, c2w[:, :3, 3:]], dim=2)
        elif c2w.shape[1:] == (4, 4):
            c2w_rdf = c2w.clone()
            c2w_rdf[:, :3, :3] = torch.einsum("nij,jk->nik", c2w[:, :3, :3], C3)
        else:
            raise ValueError(f"Unsupported c2w shape: {tuple(c2w.shape)}")
        return c2w_rdf.to(device=device, dtype=torch.float32)

    @torch.no_grad()
    def premark_invisible_cells(self, mds: List, near_plane: float = 0.05, chunk: int = 32 ** 3) -> None:
        """One-time visibility pruning: cells no camera sees get occ < 0 (HIP projection kernel)."""
        if not self.use_occ or self.occ_premarked:
            return
        mds = [md for md in mds if md is not None]
        if len(mds) == 0:
            print("[OCC] premark skipped: empty metadata list.")
            self.occ_premarked = True
            return
        device = self.occ_grid.aabbs.device
        K = self._build_intrinsics_from_metadata(mds, device)
        c2w_rdf = self._build_c2w_rdf_from_metadata(mds, device)
        H, W = int(mds[0].H), int(mds[0].W)
        self.occ_grid.mark_invisible_cells(K=K, c2w=c2w_rdf, width=W, height=H, near_plane=float(near_plane),
                                           chunk=chunk)
        self.occ_premarked = True

    @torch.no_grad()
    def maybe_update_occ_grid(self, step: int, params: Optional[Dict[str, Tensor]] = None) -> None:
        """Periodic occupancy update during training (density on the fused HIP field)."""
        if not (self.training and self.use_occ and not self.occ_frozen):
            return
        self.occ_ready = step >= self.occ_warmup_steps
        self._anneal_alpha_thre(step)

        def occ_eval_fn(x: Tensor) -> Tensor:
            return self.density(x, params=params).squeeze(-1) * self.render_step_size

        self.occ_grid.update_every_n_steps(step=step, occ_eval_fn=occ_eval_fn, occ_thre=self.occ_thre,
                                           ema_decay=self.occ_ema_decay, warmup_steps=self.occ_warmup_steps,
                                           n=self.occ_update_interval)
        self.num_occ_updates += 1
        if step % self.occ_update_interval == 0:
            print(f"[OCC UPDATE {self.num_occ_updates}] step={step:5d} warmup={step < self.occ_warmup_steps} "
                  f"alpha_thre={self.alpha_thre:6.4f}")

    @torch.no_grad()
    def _occupancy_marching_packed(self, rays: Tensor, *, params: Optional[Dict[str, Tensor]] = None,
                                   render_step_size: Optional[float] = None, alpha_thre: Optional[float] = None,
                                   cone_angle: Optional[float] = None, prefilter_aabb=None):
        """occupancy_marching plus the packed layout (chunk starts / counts per ray)."""
        if getattr(self, "occ_grid", None) is None:
            raise RuntimeError("MetaNGP: occ_grid missing")
        rays = rays.contiguous()
        o, d, t_min, t_max = rays[:, :3], rays[:, 3:6], rays[:, 6], rays[:, 7]
        sigma_fn = None
        if self.training:
            def sigma_fn(t_starts: Tensor, t_ends: Tensor, ray_indices: Tensor) -> Tensor:
                mids = 0.5 * (t_starts + t_ends)
                x = o[ray_indices] + d[ray_indices] * mids[:, None]
                return self.density(x, params=params).squeeze(-1)
        return self.occ_grid._sampling_packed(
            rays_o=o, rays_d=d, sigma_fn=sigma_fn, t_min=t_min, t_max=t_max,
            render_step_size=self.render_step_size if render_step_size is None else render_step_size,
            stratified=self.training, cone_angle=self.cone_angle if cone_angle is None else cone_angle,
            alpha_thre=self.alpha_thre if alpha_thre is None else alpha_thre, prefilter_aabb=prefilter_aabb,
            prefilter_near_far=rays[:, 6:8] if prefilter_aabb is not None else None)

    @torch.no_grad()
    def occupancy_marching(self, rays: Tensor, *, params: Optional[Dict[str, Tensor]] = None,
                           render_step_size: Optional[float] = None, alpha_thre: Optional[float] = None,
                           cone_angle: Optional[float] = None) -> Tuple[Tensor, Tensor, Tensor]:
        """(ray_indices, t_starts, t_ends) of this expert's occupied samples (meta_ngp.py:391-443)."""
        ri, t0, t1, _, _ = self._occupancy_marching_packed(rays, params=params, render_step_size=render_step_size,
                                                           alpha_thre=alpha_thre, cone_angle=cone_angle)
        return ri, t0, t1

    def get_param_groups(self) -> Dict[str, Dict]:
        return {
            "encoding": {"params": list(self.xyz_encoder.parameters())},
            "sigma": {"params": list(self.sigma_trunk.parameters()) + list(self.sigma_head.parameters())
                      + list(self.geo_head.parameters())},
            "color": {"params": list(self.color_mlp.parameters())},
        }


class _FusedMLPFn(torch.autograd.Function):
    """The expert MLP on the MFMA kernels of mlp_train.hip: forward -> [sigmoid(rgb), trunc_exp(sigma)];
    backward -> one fused kernel (acn_mlp_train_bwd_dw) that re-runs the forward of each 32-sample tile in
    registers and returns dL/d(hash features) and all 14 [dW | db] (no per-sample activations are saved).
    With DW_FUSED off, the previous split path: the forward saves the layer inputs feature-major and each
    layer's [dW | db] is one batched GEMM dY^T . [X | 1] over the batch.  First-order only: second-order
    MAML renders inside ray_rendering.second_order(), which keeps the composed torch chain."""

    DW_FUSED = True

    @staticmethod
    def forward(ctx, h0, sh, *ws):
        need = any(ctx.needs_input_grad)
        fused = _FusedMLPFn.DW_FUSED
        # the forward's packed weight image is kept for the fused backward (same weights: autograd's saved-
        # tensor version check rejects an in-place change in between), which then packs nothing itself
        prec = ops.TRAIN_MLP_PRECISION
        out, save, img = ops.mlp_train_fwd(h0, sh, ws, save=need and not fused, precision=prec, return_img=True)
        ctx.fused = fused
        ctx.prec = prec
        ctx.img = img if need and fused else None
        if need:
            if fused:
                ctx.save_for_backward(h0, sh, out, *ws)
            else:
                ctx.save_for_backward(save, out, *ws)
        return out

    @staticmethod
    def backward(ctx, g):
        need = ctx.needs_input_grad[2:]
        if ctx.fused:
            h0, sh, out, *ws = ctx.saved_tensors
            grads, gh = ops.mlp_train_bwd_dw(h0, sh, out, g.contiguous(), ws, want_h0=ctx.needs_input_grad[0],
                                             img=ctx.img, precision=ctx.prec)
            ctx.img = None
            return (gh, None, *[gr if n else None for gr, n in zip(grads, need)])
        save, out, *ws = ctx.saved_tensors
        gs, gh = ops.mlp_train_bwd(save, out, g.contiguous(), ws, want_h0=ctx.needs_input_grad[0])

        def mm(go, gn, xo, xn):  # [dW | db] of one layer: batched over the 2048-sample groups, then summed
            return torch.bmm(gs[:, go:go + gn, :], save[:, xo:xo + xn, :].transpose(1, 2)).sum(0)

        grads = [None] * 14
        if need[0] or need[1]:
            d = mm(0, 64, 0, 33)
            grads[0], grads[1] = d[:, :32], d[:, 32]
        if need[2] or need[3]:
            d = mm(64, 64, 33, 65)
            grads[2], grads[3] = d[:, :64], d[:, 64]
        if any(need[4:8]):
            d = mm(128, 16, 98, 65)
            grads[4], grads[5] = d[15:16, :64], d[15, 64:65]
            grads[6], grads[7] = d[:15, :64], d[:15, 64]
        if need[8] or need[9]:
            d = mm(144, 64, 163, 32)
            grads[8], grads[9] = d[:, :31], d[:, 31]
        if need[10] or need[11]:
            d = mm(208, 64, 195, 65)
            grads[10], grads[11] = d[:, :64], d[:, 64]
        if need[12] or need[13]:
            d = mm(272, 3, 260, 65)
            grads[12], grads[13] = d[:, :64], d[:, 64]
        grads = [gr if n else None for gr, n in zip(grads, need)]
        return (gh, None, *grads)
