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


@pytest.mark.parametrize("n", [1, 4113, 300_007])
def test_fused_dw_matches_split_path(n):
    """acn_mlp_train_bwd_dw (forward re-run in registers, [dW | db] on MFMA, workgroup partials) against
    the split path (saved activations + batched GEMMs): dL/dh0 and all 14 gradients.  n = 300k fills
    every partial slot (256 workgroups x 4 waves x > 1 tile)."""
    from adaptive_city_nerf_amd import ops
    g = torch.Generator(device="cuda").manual_seed(n)
    sub = _expert()
    ws = [t.detach().contiguous() for t in (
        sub.sigma_trunk[0].linear.weight, sub.sigma_trunk[0].linear.bias, sub.sigma_trunk[1].linear.weight,
        sub.sigma_trunk[1].linear.bias, sub.sigma_head.weight, sub.sigma_head.bias, sub.geo_head.weight,
        sub.geo_head.bias, sub.color_mlp[0].linear.weight, sub.color_mlp[0].linear.bias,
        sub.color_mlp[1].linear.weight, sub.color_mlp[1].linear.bias, sub.color_mlp[2].weight,
        sub.color_mlp[2].bias)]
    h0 = (torch.rand(n, 32, device="cuda", generator=g) - 0.5) * 2
    sh = (torch.rand(n, 16, device="cuda", generator=g) - 0.5) * 2
    gout = torch.randn(n, 4, device="cuda", generator=g)
    out, save = ops.mlp_train_fwd(h0, sh, ws, save=True)
    out2, _ = ops.mlp_train_fwd(h0, sh, ws, save=False)
    assert torch.equal(out, out2)
    fused, gh_f = ops.mlp_train_bwd_dw(h0, sh, out, gout, ws, want_h0=True)
    gs, gh_s = ops.mlp_train_bwd(save, out, gout, ws, want_h0=True)
    # split path: layer GEMMs over the saved feature-major blocks
    mm = lambda go, gn, xo, xn: torch.bmm(gs[:, go:go + gn, :].double(),  # noqa: E731
                                          save[:, xo:xo + xn, :].double().transpose(1, 2)).sum(0)
    d0, d1, dh, dc0, dc1, dc2 = mm(0, 64, 0, 33), mm(64, 64, 33, 65), mm(128, 16, 98, 65), mm(144, 64, 163, 32), \
        mm(208, 64, 195, 65), mm(272, 3, 260, 65)
    split = [d0[:, :32], d0[:, 32], d1[:, :64], d1[:, 64], dh[15:16, :64], dh[15, 64:65], dh[:15, :64], dh[:15, 64],
             dc0[:, :31], dc0[:, 31], dc1[:, :64], dc1[:, 64], dc2[:, :64], dc2[:, 64]]
    assert torch.equal(gh_f, gh_s)  # same chain, same order: bit-identical
    for k, (a, b) in enumerate(zip(fused, split)):
        assert a.shape == b.shape, (k, a.shape, b.shape)
        a, b = a.double().cpu().numpy(), b.cpu().numpy()
        scale = max(np.abs(b).max(), 1e-12)
        assert np.abs(a - b).max() <= 2e-5 * scale + 1e-9, (k, np.abs(a - b).max(), scale)


@pytest.mark.parametrize("precision", ["fp16x3", "fp32"])
def test_fused_dw_on_forward_image(precision):
    """acn_mlp_train_bwd_dw_img (the backward on the image the forward packed, no pack of its own) against
    acn_mlp_train_bwd_dw (its own pack of the same weights): the same kernels on the same image."""
    from adaptive_city_nerf_amd import ops
    n = 4113
    g = torch.Generator(device="cuda").manual_seed(11)
    sub = _expert()
    ws = [t.detach().contiguous() for t in (
        sub.sigma_trunk[0].linear.weight, sub.sigma_trunk[0].linear.bias, sub.sigma_trunk[1].linear.weight,
        sub.sigma_trunk[1].linear.bias, sub.sigma_head.weight, sub.sigma_head.bias, sub.geo_head.weight,
        sub.geo_head.bias, sub.color_mlp[0].linear.weight, sub.color_mlp[0].linear.bias,
        sub.color_mlp[1].linear.weight, sub.color_mlp[1].linear.bias, sub.color_mlp[2].weight,
        sub.color_mlp[2].bias)]
    h0 = (torch.rand(n, 32, device="cuda", generator=g) - 0.5) * 2
    sh = (torch.rand(n, 16, device="cuda", generator=g) - 0.5) * 2
    gout = torch.randn(n, 4, device="cuda", generator=g)
    out, _, img = ops.mlp_train_fwd(h0, sh, ws, save=False, precision=precision, return_img=True)
    a, gha = ops.mlp_train_bwd_dw(h0, sh, out, gout, ws, want_h0=True, precision=precision)
    b, ghb = ops.mlp_train_bwd_dw(h0, sh, out, gout, ws, want_h0=True, img=img, precision=precision)
    assert torch.equal(gha, ghb)
    for x, y in zip(a, b):
        scale = max(float(x.abs().max()), 1e-12)
        assert float((x - y).abs().max()) <= 1e-6 * scale


def test_fused_dw_empty_batch():
    from adaptive_city_nerf_amd import ops
    z = torch.zeros(0, 32, device="cuda")
    out = torch.zeros(0, 4, device="cuda")
    ws14 = [torch.zeros(s, device="cuda") for s in ops.MLP_DW_SHAPES]
    grads, gh = ops.mlp_train_bwd_dw(z, torch.zeros(0, 16, device="cuda"), out, out, ws14, want_h0=True)
    assert gh.shape == (0, 32) and all(float(g.abs().max()) == 0.0 for g in grads)


def test_split_path_still_matches_composed():
    """The previous split backward stays selectable (_FusedMLPFn.DW_FUSED = False) and correct."""
    from adaptive_city_nerf_amd.meta_ngp import _FusedMLPFn
    old = _FusedMLPFn.DW_FUSED
    _FusedMLPFn.DW_FUSED = False
    try:
        test_fused_mlp_matches_composed(1000)
    finally:
        _FusedMLPFn.DW_FUSED = old


@pytest.mark.parametrize("wscale,gscale,tscale", [(1.0, 1e-10, 1.0), (1.0, 1e6, 1.0), (12.0, 1.0, 1.0),
                                                  (1.0, 1e-8, 0.005)])
def test_fused_mlp_extreme_ranges(wscale, gscale, tscale):
    """The fp16x3 layers' per-layer power-of-two scaling (mlp_train.hip): output gradients of 1e-10 or 1e6,
    activations pushed past fp16's 65504 by large weights, and hash features at the reference's default
    table scale (|h0| ~ 1e-3): outputs and gradients still match the composed fp32 chain."""
    from adaptive_city_nerf_amd.ray_rendering import second_order
    sub = _expert()
    with torch.no_grad():
        for n_, p in sub.named_parameters():
            if n_.endswith("hash_table"):
                p.mul_(tscale)
            elif "weight" in n_:
                p.mul_(wscale)
    n = 2048
    xd = _inputs(sub, n, 11)
    gw = gscale * torch.randn(n, 4, device="cuda", generator=torch.Generator(device="cuda").manual_seed(5))
    params = list(sub.parameters())
    out_f = sub(xd)
    gf = torch.autograd.grad((out_f * gw).sum(), params, allow_unused=True)
    with second_order():
        out_c = sub(xd)
        gc = torch.autograd.grad((out_c * gw).sum(), params, allow_unused=True)
    # large weights make every layer's sum cancel: the split keeps ~2^-22 per product against fp32's
    # 2^-24 per fma, so the ill-conditioned case gets a correspondingly wider bound
    tol = 2e-5 if wscale == 1.0 else 2e-4
    a, b = out_f.detach().double().cpu().numpy(), out_c.detach().double().cpu().numpy()
    scale_o = np.maximum(np.abs(b).max(axis=0), 1e-30)
    assert np.isfinite(a).all()
    assert (np.abs(a - b) / scale_o).max() <= tol
    for (name, _), x, y in zip(sub.named_parameters(), gf, gc):
        if y is None:
            continue
        x, y = x.detach().double().cpu().numpy(), y.detach().double().cpu().numpy()
        scale = max(np.abs(y).max(), 1e-300)
        assert np.isfinite(x).all(), name
        assert np.abs(x - y).max() <= 2.5 * tol * scale, (name, np.abs(x - y).max(), scale)
