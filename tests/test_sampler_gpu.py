"""Training-path sampler (acn_sample_stratified, ray_rendering.render_rays_stratified's differentiable
single-expert branch) against the composed torch chain it replaces: stratified_t_vals
(ray_rendering.py:262-287), o + d t, MetaNGP._world_to_unit (meta_ngp.py:155-158) and the colour-branch
SH (meta_ngp.py:165-168) bit for bit; renders and gradients against the composed path."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _model():
    from test_module_api import build_model
    m, _ = build_model("k4")
    m = m.cuda().train()
    g = torch.Generator().manual_seed(3)
    with torch.no_grad():
        for sub in m.submodules:
            for p in sub.meta_parameters():
                p.copy_((torch.rand(p.shape, generator=g) - 0.5) * 0.4)
            t = sub.xyz_encoder.hash_table
            t.copy_((torch.rand(t.shape, generator=g) - 0.5) * 0.2)
    return m


def _rays(sub, n, seed, degenerate=False):
    g = torch.Generator(device="cuda").manual_seed(seed)
    mn, mx = sub.scene_box.min.cuda(), sub.scene_box.max.cuda()
    o = mn + (mx - mn) * torch.rand(n, 3, device="cuda", generator=g)
    d = torch.randn(n, 3, device="cuda", generator=g)
    if degenerate:
        d[::7] = 0.0          # zero direction: norm clamp
        d[1::7, 1:] = 0.0     # axis-parallel
    near = 0.05 * torch.rand(n, device="cuda", generator=g)
    far = near + torch.rand(n, device="cuda", generator=g)
    return torch.cat([o, d, near[:, None], far[:, None]], 1).contiguous()


@pytest.mark.parametrize("S,degenerate", [(96, False), (1, False), (2, True), (257, True)])
def test_sampler_bitwise_vs_reference_ops(S, degenerate):
    """The reference's own ops, evaluated on the CPU (its parity device): t-values, points, unit-box
    coordinates; the SH rows equal the HIP SH encoder (bit-exact vs the reference) of the CPU-normalised
    directions, i.e. _enc_dir's two normalisations."""
    from adaptive_city_nerf_amd import ops
    from adaptive_city_nerf_amd.ray_rendering import stratified_t_vals
    sub = _model().submodules[1]
    rays = _rays(sub, 777, S, degenerate)
    u = torch.rand(777, S, device="cuda", generator=torch.Generator(device="cuda").manual_seed(5))
    mn, ext = sub._host_box()
    rc = rays.cpu()
    for jit in (u, None):
        t, x01, sh = ops.sample_stratified(rays, S, jit, mn, ext, 1e-6)
        t_ref = stratified_t_vals(rc[:, 6], rc[:, 7], S, randomized=jit is not None,
                                  u=None if jit is None else jit.cpu())
        assert torch.equal(t.cpu(), t_ref)
        pts = rc[:, None, :3] + rc[:, None, 3:6] * t_ref[..., None]
        eps = sub.enc_eps.cpu()
        x_ref = ((pts.reshape(-1, 3) - torch.tensor(mn)) / torch.tensor(ext)).clamp(eps, 1.0 - eps)
        assert torch.equal(x01.cpu(), x_ref)
        d = rc[:, 3:6]
        dn = d / d.norm(dim=-1, keepdim=True).clamp_min_(1e-9)
        sh_ray = ops.sh_fwd(dn.cuda(), 4).cpu()
        sh_ref = sh_ray[:, None, :].expand(-1, S, -1).reshape(-1, 16)
        assert torch.equal(torch.nan_to_num(sh.cpu(), 7.0), torch.nan_to_num(sh_ref, 7.0))


def test_training_render_matches_composed_chain():
    """render_rays in training mode (jitter given, active_module): the fused sampler branch against the
    composed chain on the GPU (whose torch norm / division may round differently from the CPU reference
    the sampler follows): outputs and parameter gradients within fp32 tolerance."""
    from adaptive_city_nerf_amd import ray_rendering as RR
    m = _model()
    rays = _rays(m.submodules[2], 1000, 11)
    u = torch.rand(1000, 96, device="cuda", generator=torch.Generator(device="cuda").manual_seed(2))
    tgt = torch.rand(1000, 3, device="cuda", generator=torch.Generator(device="cuda").manual_seed(4))
    res = []
    for fused in (True, False):
        RR.FUSED_TRAIN_SAMPLER = fused
        try:
            m.zero_grad(set_to_none=True)
            rgb, depth, w, acc = RR.render_rays(m, rays, ray_samples=96, active_module=2, jitter_u=u,
                                                bg_color_default="white")
            ((rgb - tgt) ** 2).mean().backward()
            res.append(([x.detach().clone() for x in (rgb, depth, w, acc)],
                        {n: p.grad.detach().clone() for n, p in m.named_parameters() if p.grad is not None}))
        finally:
            RR.FUSED_TRAIN_SAMPLER = True
    (o_f, g_f), (o_c, g_c) = res
    for a, b in zip(o_f, o_c):
        assert float((a - b).abs().max()) <= 1e-5
    assert g_f.keys() == g_c.keys()
    for k in g_f:
        a, b = g_f[k].double().cpu().numpy(), g_c[k].double().cpu().numpy()
        scale = max(np.abs(b).max(), 1e-12)
        assert np.abs(a - b).max() <= 1e-5 * scale + 1e-12, (k, np.abs(a - b).max(), scale)
