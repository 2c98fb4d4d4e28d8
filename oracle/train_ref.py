"""CPU restatement of the reference's online-adaptation step -- TEST INFRASTRUCTURE ONLY.

A plain-PyTorch (CPU, fp32) re-statement of the path one ``runtime_adapt`` update runs
(pipelines/online_stage/runtime_adapt.py:288-313): stratified samples (nerfs/ray_rendering.py:
262-287, with the jitter uniforms supplied) -> MetaContainer soft routing (models/inr/
meta_container.py:97-134, 275-343) -> per-expert MetaNGP (models/inr/meta_ngp.py:155-241: hash grid
models/encodings.py:308-381, MLPs, trunc_exp models/trunc_exp.py:30-61, SH encodings.py:27-81) ->
background head (meta_container.py:347-382) -> volume_render (ray_rendering.py:114-165) ->
compute_mse_loss (nerfs/losses.py:10-32, color_space.py:22-66) -> backward -> clip_grad_norm_ ->
torch.optim.Adam param groups (common/utils.py:16-62).

Only tests/ and bench.py's cpu_baseline leg import this module, as the checker / CPU baseline of
the HIP training step; the product package never does.  It is pinned by tests/golden/train_k4.npz
(generated from the reference itself): tests/test_oracle_golden.py::test_train_ref_matches_fixture.
Parameters use the reference's state-dict names.
"""
from __future__ import annotations

from typing import Dict, List, Optional

import numpy as np
import torch
import torch.nn.functional as F

PRIMES = (1, 2654435761, 805459861)
SH_C = (0.28209479177387814, 0.4886025119029199, 1.0925484305920792, 0.9461746957575601, 0.31539156525251999,
        0.5462742152960396, 0.5900435899266435, 2.890611442640554, 0.4570457994644658, 0.3731763325901154,
        1.445305721320277)


class _TruncExp(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        xc = x.clamp(-88.722839111, 88.722839111)
        ctx.save_for_backward(xc)
        return torch.exp(xc)

    @staticmethod
    def backward(ctx, g):
        (xc,) = ctx.saved_tensors
        return g * torch.exp(xc)


def sh_deg3(d: torch.Tensor) -> torch.Tensor:
    """16 real SH components of unit directions (encodings.py:27-81, levels=4)."""
    x, y, z = d[..., 0], d[..., 1], d[..., 2]
    xx, yy, zz = x * x, y * y, z * z
    c = SH_C
    comps = [torch.full_like(x, c[0]), c[1] * y, c[1] * z, c[1] * x,
             c[2] * x * y, c[2] * y * z, c[3] * zz - c[4], c[2] * x * z, c[5] * (xx - yy),
             c[6] * y * (3 * xx - yy), c[7] * x * y * z, c[8] * y * (5 * zz - 1), c[9] * z * (5 * zz - 3),
             c[8] * x * (5 * zz - 1), c[10] * z * (xx - yy), c[6] * x * (xx - 3 * yy)]
    return torch.stack(comps, dim=-1)


def sh_enc(d: torch.Tensor) -> torch.Tensor:
    """SHEncoder.forward (encodings.py:133-151): normalise (clamp 1e-9), then the components."""
    return sh_deg3(d / d.norm(dim=-1, keepdim=True).clamp_min(1e-9))


def hash_encode(x01: torch.Tensor, table: torch.Tensor, res: torch.Tensor, log2T: int) -> torch.Tensor:
    """Multiresolution hash grid, trilinear, x -> y -> z lerp order (encodings.py:308-381)."""
    L = res.shape[0]
    T = 1 << log2T
    offsets = torch.arange(L, dtype=torch.int64) * T
    scaled = x01[..., None, :] * res.to(x01.dtype).view(1, L, 1)
    fl = torch.floor(scaled)
    frac = scaled - fl
    fl = fl.to(torch.int64)
    ce = fl + 1

    def gather(ix, iy, iz):
        idx = ((ix * PRIMES[0]) ^ (iy * PRIMES[1]) ^ (iz * PRIMES[2])) % T
        return table[idx + offsets]

    f000 = gather(fl[..., 0], fl[..., 1], fl[..., 2]); f001 = gather(fl[..., 0], fl[..., 1], ce[..., 2])
    f010 = gather(fl[..., 0], ce[..., 1], fl[..., 2]); f011 = gather(fl[..., 0], ce[..., 1], ce[..., 2])
    f100 = gather(ce[..., 0], fl[..., 1], fl[..., 2]); f101 = gather(ce[..., 0], fl[..., 1], ce[..., 2])
    f110 = gather(ce[..., 0], ce[..., 1], fl[..., 2]); f111 = gather(ce[..., 0], ce[..., 1], ce[..., 2])
    wx, wy, wz = frac[..., 0:1], frac[..., 1:2], frac[..., 2:3]
    c00 = f000 * (1 - wx) + f100 * wx
    c01 = f001 * (1 - wx) + f101 * wx
    c10 = f010 * (1 - wx) + f110 * wx
    c11 = f011 * (1 - wx) + f111 * wx
    c0 = c00 * (1 - wy) + c10 * wy
    c1 = c01 * (1 - wy) + c11 * wy
    return (c0 * (1 - wz) + c1 * wz).flatten(start_dim=-2)


class RefContainer:
    """Parameters (reference state-dict names) + forward of MetaContainer with MetaNGP experts."""

    def __init__(self, state: Dict[str, torch.Tensor], K: int, res: np.ndarray, log2T: int, centroids, bm: float,
                 mins, extents, cluster_2d: bool = True):
        self.p = {k: v.detach().clone().float().requires_grad_(k.endswith(("weight", "bias", "hash_table")))
                  for k, v in state.items()}
        self.K, self.log2T, self.bm, self.cluster_2d = K, log2T, float(bm), cluster_2d
        self.res = torch.as_tensor(np.asarray(res), dtype=torch.int64)
        self.cent = torch.as_tensor(np.asarray(centroids), dtype=torch.float32)
        self.mins = torch.as_tensor(np.asarray(mins), dtype=torch.float32)
        self.ext = torch.as_tensor(np.asarray(extents), dtype=torch.float32)

    def param_groups(self, lrs: Dict[str, float], K_active: Optional[List[int]] = None):
        g = {"encoding": [], "sigma": [], "color": [], "background": []}
        for k in range(self.K):
            pre = f"submodules.{k}."
            g["encoding"].append(self.p[pre + "xyz_encoder.hash_table"])
            for n in ("sigma_trunk.0.linear", "sigma_trunk.1.linear", "sigma_head", "geo_head"):
                g["sigma"] += [self.p[pre + n + ".weight"], self.p[pre + n + ".bias"]]
            for n in ("color_mlp.0.linear", "color_mlp.1.linear", "color_mlp.2"):
                g["color"] += [self.p[pre + n + ".weight"], self.p[pre + n + ".bias"]]
        g["background"] = [self.p[f"bg_mlp.{i}.{w}"] for i in (0, 2) for w in ("weight", "bias")]
        return [{"params": v, "lr": lrs[n], "name": n} for n, v in g.items()]

    def parameters(self):
        return [v for v in self.p.values() if v.requires_grad]

    def expert(self, k: int, x_d: torch.Tensor) -> torch.Tensor:
        p, pre = self.p, f"submodules.{k}."
        x, d = x_d[:, :3], x_d[:, 3:6]
        x01 = ((x - self.mins[k]) / self.ext[k]).clamp(1e-6, 1.0 - 1e-6)
        h = hash_encode(x01, p[pre + "xyz_encoder.hash_table"], self.res, self.log2T)
        for i in (0, 1):
            h = F.relu(h.matmul(p[pre + f"sigma_trunk.{i}.linear.weight"].t()) + p[pre + f"sigma_trunk.{i}.linear.bias"])
        sigma = _TruncExp.apply(h.matmul(p[pre + "sigma_head.weight"].t()) + p[pre + "sigma_head.bias"])
        geo = h.matmul(p[pre + "geo_head.weight"].t()) + p[pre + "geo_head.bias"]
        dn = d / d.norm(dim=-1, keepdim=True).clamp_min(1e-9)
        c = torch.cat([geo, sh_enc(dn)], dim=-1)
        for i in (0, 1):
            c = F.relu(c.matmul(p[pre + f"color_mlp.{i}.linear.weight"].t()) + p[pre + f"color_mlp.{i}.linear.bias"])
        rgb = torch.sigmoid(c.matmul(p[pre + "color_mlp.2.weight"].t()) + p[pre + "color_mlp.2.bias"])
        return torch.cat([rgb, sigma], dim=-1)

    def forward(self, x: torch.Tensor, active_module: Optional[int] = None) -> torch.Tensor:
        if active_module is not None:
            return self.expert(active_module, x)
        idx = [1, 2] if self.cluster_2d else [0, 1, 2]
        with torch.no_grad():
            dist = torch.cdist(x[:, idx].float(), self.cent[:, idx].float()).clamp_min(1e-6)
            invd = 1.0 / dist
            mind = dist.min(dim=1, keepdim=True).values
            invd = invd * (dist <= self.bm * mind)
            w = invd / invd.sum(dim=1, keepdim=True).clamp_min(1e-6)
        out = None
        for k in range(self.K):
            sel = (w[:, k] > 0).nonzero(as_tuple=False).squeeze(1)
            if sel.numel() == 0:
                continue
            yk = self.expert(k, x.index_select(0, sel))
            if out is None:
                out = x.new_zeros(x.shape[0], yk.shape[-1])
            out.index_add_(0, sel, yk * w[:, k].index_select(0, sel).unsqueeze(1))
        return out if out is not None else x.new_zeros(x.shape[0], 4)

    def background(self, d: torch.Tensor) -> torch.Tensor:
        p = self.p
        enc = sh_enc(F.normalize(d, dim=-1))
        h = F.relu(enc.matmul(p["bg_mlp.0.weight"].t()) + p["bg_mlp.0.bias"])
        return torch.sigmoid(h.matmul(p["bg_mlp.2.weight"].t()) + p["bg_mlp.2.bias"])


def render_train(model: RefContainer, rays: torch.Tensor, S: int, u: torch.Tensor, active_module=None):
    o, d = rays[:, :3], rays[:, 3:6]
    near, far = rays[:, 6], rays[:, 7]
    t_lin = torch.linspace(0.0, 1.0, S).unsqueeze(0)
    t = near.unsqueeze(1) * (1.0 - t_lin) + far.unsqueeze(1) * t_lin
    mids = 0.5 * (t[:, :-1] + t[:, 1:])
    low = torch.cat([t[:, :1], mids], 1)
    high = torch.cat([mids, t[:, -1:]], 1)
    t = low + (high - low) * u
    pts = o.unsqueeze(1) + d.unsqueeze(1) * t.unsqueeze(-1)
    dirs = d.unsqueeze(1).expand_as(pts)
    rs = model.forward(torch.cat([pts, dirs], -1).reshape(-1, 6), active_module).view(pts.shape[0], S, 4)
    bg = model.background(dirs[:, 0])
    rgb = rs[..., :3].clamp(0.0, 1.0)
    sigma = rs[..., 3].clamp_min(0.0)
    dists = (t[:, 1:] - t[:, :-1]).clamp_min(1e-4)
    dists = torch.cat([dists, dists[:, -1:]], 1)
    alpha = (1.0 - torch.exp(-sigma * dists)).clamp(0.0, 1.0 - 1e-7)
    T = torch.cumprod(torch.cat([torch.ones_like(alpha[:, :1]), 1.0 - alpha + 1e-10], 1), 1)[:, :-1]
    w = alpha * T
    acc = w.sum(1)
    return (w.unsqueeze(-1) * rgb).sum(1) + (1.0 - acc.unsqueeze(-1)) * bg


def srgb_to_linear(x):
    return torch.where(x <= 0.04045, x / 12.92, ((x + 0.055) / 1.055).pow(2.4))


def adapt_step(model: RefContainer, opt, rays, rgbs, S, u, active_module=None, clip=1.0):
    """One runtime_adapt update; returns (loss, total_norm_before_clip, {name: grad copy})."""
    opt.zero_grad()
    pred = render_train(model, rays, S, u, active_module)
    loss = F.mse_loss(pred.clamp(0, 1), srgb_to_linear(rgbs.clamp(0, 1)).clamp(0, 1))
    loss.backward()
    grads = {k: (None if v.grad is None else v.grad.detach().clone()) for k, v in model.p.items() if v.requires_grad}
    tn = torch.nn.utils.clip_grad_norm_([v for v in model.parameters() if v.grad is not None], clip)
    opt.step()
    return float(loss.detach()), float(tn), grads
