"""The training-path expert MLP on MFMA (mlp_train.hip, meta_ngp._FusedMLPFn) against the composed torch
chain it replaces (the path second-order MAML keeps): outputs and every gradient (hash table, the 14
MLP tensors, fast weights) within fp32 GEMM-reordering tolerance."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _expert():
    from test_module_api import build_model
    m, _ = build_model("k1")
    sub = m.submodules[0].cuda().train()
    g = torch.Generator().manual_seed(0)
    with torch.no_grad():
        for p in sub.meta_parameters():
            p.copy_((torch.rand(p.shape, generator=g) - 0.5) * 0.4)
    return sub


def _inputs(sub, n, seed):
    g = torch.Generator(device="cuda").manual_seed(seed)
    mn, mx = sub.scene_box.min.cuda(), sub.scene_box.max.cuda()
    x = mn + (mx - mn) * torch.rand(n, 3, device="cuda", generator=g)
    d = torch.nn.functional.normalize(torch.randn(n, 3, device="cuda", generator=g), dim=-1)
    return torch.cat([x, d], -1)


@pytest.mark.parametrize("n", [1, 31, 1000, 4096 + 17])
def test_fused_mlp_matches_composed(n):
    from adaptive_city_nerf_amd.ray_rendering import second_order
    sub = _expert()
    xd = _inputs(sub, n, n)
    gw = torch.rand(n, 4, device="cuda", generator=torch.Generator(device="cuda").manual_seed(1))
    params = list(sub.parameters())
    out_f = sub(xd)
    gf = torch.autograd.grad((out_f * gw).sum(), params, allow_unused=True)
    with second_order():
        out_c = sub(xd)
        gc = torch.autograd.grad((out_c * gw).sum(), params, allow_unused=True)
    np.testing.assert_allclose(out_f.detach().cpu().numpy(), out_c.detach().cpu().numpy(), rtol=1e-5, atol=1e-6)
    for (name, _), a, b in zip(sub.named_parameters(), gf, gc):
        if b is None:
            assert a is None or float(a.abs().max()) == 0.0, name
            continue
        a, b = a.detach().double().cpu().numpy(), b.detach().double().cpu().numpy()
        scale = max(np.abs(b).max(), 1e-12)
        assert np.abs(a - b).max() <= 2e-5 * scale + 1e-9, (name, np.abs(a - b).max(), scale)


def test_fused_mlp_fast_weights():
    """Fast weights (MAML params dicts) take the fused path too and get gradients."""
    sub = _expert()
    xd = _inputs(sub, 700, 3)
    fast = {k: v.detach().clone().requires_grad_(True) for k, v in sub.meta_named_parameters()}
    out = sub(xd, params=fast)
    g = torch.autograd.grad(out.square().sum(), list(fast.values()))
    assert all(t is not None and torch.isfinite(t).all() for t in g)
