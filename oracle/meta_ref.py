"""CPU restatement of the reference's offline meta-training step -- TEST INFRASTRUCTURE ONLY.

Plain PyTorch (CPU, fp32) over train_ref.RefContainer: pipelines/offline_stage/meta_core.py
(task_adapt :14-67 with fast weights resolved like MetaModule.get_subdict, maml_meta_update
:126-143, reptile_meta_update :146-182) and meta_train_step.py:18-253 (region order, per-task inner
loop on the support set, query loss with the adapted weights, sample-weighted region sums, FedAvg
scaling by the number of regions), compute_mse_loss (nerfs/losses.py:10-32) in linear colour space.
The expert render with ``active_module`` keeps the container's background head, as
render_rays_stratified does (ray_rendering.py:330-345).  Only tests/ import this module; it is
pinned by tests/golden/meta_{fomaml,maml,reptile}.npz (generated from the reference itself).
"""
from __future__ import annotations

from collections import OrderedDict
from typing import Dict, Iterator, List, Sequence

import torch
import torch.nn.functional as F

from .train_ref import RefContainer, _TruncExp, hash_encode, sh_enc, srgb_to_linear

MLP_NAMES = ("sigma_trunk.0.linear.weight", "sigma_trunk.0.linear.bias", "sigma_trunk.1.linear.weight",
             "sigma_trunk.1.linear.bias", "sigma_head.weight", "sigma_head.bias", "geo_head.weight", "geo_head.bias",
             "color_mlp.0.linear.weight", "color_mlp.0.linear.bias", "color_mlp.1.linear.weight",
             "color_mlp.1.linear.bias", "color_mlp.2.weight", "color_mlp.2.bias")


def expert_fast(m: RefContainer, k: int, x_d: torch.Tensor, fast: Dict[str, torch.Tensor]) -> torch.Tensor:
    """MetaNGP.forward of expert k with the fast weights (expert-relative names) (meta_ngp.py:171-241)."""
    p, pre = m.p, f"submodules.{k}."
    W = lambda n: fast[n] if n in fast else p[pre + n]  # noqa: E731
    x, d = x_d[:, :3], x_d[:, 3:6]
    x01 = ((x - m.mins[k]) / m.ext[k]).clamp(1e-6, 1.0 - 1e-6)
    h = hash_encode(x01, p[pre + "xyz_encoder.hash_table"], m.res, m.log2T)
    for i in (0, 1):
        h = F.relu(h.matmul(W(f"sigma_trunk.{i}.linear.weight").t()) + W(f"sigma_trunk.{i}.linear.bias"))
    sigma = _TruncExp.apply(h.matmul(W("sigma_head.weight").t()) + W("sigma_head.bias"))
    geo = h.matmul(W("geo_head.weight").t()) + W("geo_head.bias")
    dn = d / d.norm(dim=-1, keepdim=True).clamp_min(1e-9)
    c = torch.cat([geo, sh_enc(dn)], dim=-1)
    for i in (0, 1):
        c = F.relu(c.matmul(W(f"color_mlp.{i}.linear.weight").t()) + W(f"color_mlp.{i}.linear.bias"))
    rgb = torch.sigmoid(c.matmul(W("color_mlp.2.weight").t()) + W("color_mlp.2.bias"))
    return torch.cat([rgb, sigma], dim=-1)


def render_fast(m: RefContainer, rays, S: int, u, k: int, fast) -> torch.Tensor:
    """Training-mode render_rays(model, rays, params=fast, active_module=k): rgb (N, 3)."""
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
    rs = expert_fast(m, k, torch.cat([pts, dirs], -1).reshape(-1, 6), fast).view(pts.shape[0], S, 4)
    bg = m.background(dirs[:, 0])
    rgb = rs[..., :3].clamp(0.0, 1.0)
    sigma = rs[..., 3].clamp_min(0.0)
    dists = (t[:, 1:] - t[:, :-1]).clamp_min(1e-4)
    dists = torch.cat([dists, dists[:, -1:]], 1)
    alpha = (1.0 - torch.exp(-sigma * dists)).clamp(0.0, 1.0 - 1e-7)
    T = torch.cumprod(torch.cat([torch.ones_like(alpha[:, :1]), 1.0 - alpha + 1e-10], 1), 1)[:, :-1]
    w = alpha * T
    acc = w.sum(1)
    return (w.unsqueeze(-1) * rgb).sum(1) + (1.0 - acc.unsqueeze(-1)) * bg


def mse_linear(pred, gt):
    return F.mse_loss(pred.clamp(0, 1), srgb_to_linear(gt.clamp(0, 1)).clamp(0, 1))


def task_adapt(m: RefContainer, support, S: int, us: Iterator[torch.Tensor], inner_lr: float, iters: int, k: int,
               algo: str):
    first_order = algo in ("fomaml", "reptile")
    if algo == "reptile":
        fast = OrderedDict((n, m.p[f"submodules.{k}.{n}"].detach().clone().requires_grad_(True)) for n in MLP_NAMES)
    else:
        fast = OrderedDict((n, m.p[f"submodules.{k}.{n}"]) for n in MLP_NAMES)
    losses = []
    for _ in range(iters):
        loss = mse_linear(render_fast(m, support["rays"], S, next(us), k, fast), support["rgbs"])
        grads = torch.autograd.grad(loss, tuple(fast.values()), create_graph=not first_order, allow_unused=True)
        fast = OrderedDict((n, w if g is None else w - inner_lr * g) for (n, w), g in zip(fast.items(), grads))
        losses.append(loss.detach())
    return fast, losses


def meta_step(m: RefContainer, opt, task_data, order: Sequence[int], S: int, us: Iterator[torch.Tensor],
              algo: str, inner_lr: float, inner_iter: int, lr: float, clip: float = 1.0):
    """One train_step (maml / fomaml) or the Reptile update rule over the same tasks."""
    if algo == "reptile":
        fast_list: List[Dict[str, torch.Tensor]] = []
        for cid in order:
            fast, _ = task_adapt(m, task_data[cid]["support"], S, us, inner_lr, inner_iter, cid, algo)
            fast_list.append({f"submodules.{cid}.{n}": v for n, v in fast.items()})
        with torch.no_grad():
            for name in [f"submodules.{cid}.{n}" for cid in order for n in MLP_NAMES]:
                delta = sum(f[name].detach() - m.p[name].detach() for f in fast_list if name in f) / len(fast_list)
                if torch.isfinite(delta).all() and delta.abs().sum() > 0:
                    m.p[name].add_(lr * delta)
        return None
    q_sum, q_cnt = 0.0, 0
    for cid in order:
        sup, qry = task_data[cid]["support"], task_data[cid]["query"]
        fast, _ = task_adapt(m, sup, S, us, inner_lr, inner_iter, cid, algo)
        loss_q = mse_linear(render_fast(m, qry["rays"], S, next(us), cid, fast), qry["rgbs"])
        q_sum = q_sum + loss_q * qry["rays"].shape[0]
        q_cnt += qry["rays"].shape[0]
    loss_meta = len(order) * (q_sum / q_cnt)
    opt.zero_grad(set_to_none=True)
    loss_meta.backward()
    params = [p for g in opt.param_groups for p in g["params"] if p.grad is not None]
    torch.nn.utils.clip_grad_norm_(params, clip)
    opt.step()
    return float(loss_meta.detach())
