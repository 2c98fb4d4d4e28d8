"""Deterministic hash-grid backward (acn_hashgrid_bwd_det): against a serial CPU scatter-add.

The serial restatement below adds every (point, level, corner) gradient to its table row in point
order in fp32 (np.add.at is sequential), i.e. what a CPU loop over the points does (the reference's
index_put_(accumulate=True) backward, models/encodings.py:318-329, on the CPU).  It is first checked
against the reference's own gradient fixtures (tests/golden/hashgrid.npz); the GPU deterministic
mode must then equal it BIT FOR BIT, be bitwise reproducible run to run, and be what autograd runs
under torch.use_deterministic_algorithms(True).
"""
import numpy as np
import pytest
import torch

import goldens as G

P1, P2 = np.uint32(2654435761), np.uint32(805459861)


def serial_scatter(x01, gout, res, L, log2T, interp):
    """(L * 2^log2T, 2) fp32 table gradient, rows summed in (point, corner) order."""
    x01 = np.asarray(x01, np.float32)
    M = x01.shape[0]
    T = 1 << log2T
    mask = np.uint32(T - 1)
    g = np.asarray(gout, np.float32).reshape(M, L, 2)
    keys, vals = [], []
    with np.errstate(over="ignore"):
        s = x01[:, None, :] * np.asarray(res, np.float32)[None, :, None]          # (M, L, 3)
        if interp == 0:
            ix = np.rint(s).astype(np.int64).astype(np.uint32)
            h = (ix[..., 0] ^ (ix[..., 1] * P1) ^ (ix[..., 2] * P2)) & mask
            keys = (np.arange(L, dtype=np.uint64)[None, :] * T + h).reshape(-1)
            vals = g.reshape(-1, 2)
        else:
            f = np.floor(s)
            w = (s - f).astype(np.float32)
            if interp == 2:
                w = ((w * w) * (np.float32(3.0) - np.float32(2.0) * w)).astype(np.float32)
            a = (np.float32(1.0) - w).astype(np.float32)
            i0 = f.astype(np.int64).astype(np.uint32)
            k_all, v_all = np.empty((M, L, 8), np.uint64), np.empty((M, L, 8, 2), np.float32)
            for c in range(8):
                bx, by, bz = c >> 2, (c >> 1) & 1, c & 1
                h = ((i0[..., 0] + np.uint32(bx)) ^ (i0[..., 1] * P1 + (P1 if by else np.uint32(0)))
                     ^ (i0[..., 2] * P2 + (P2 if bz else np.uint32(0)))) & mask
                k_all[..., c] = np.arange(L, dtype=np.uint64)[None, :] * T + h
                fz = w[..., 2] if bz else a[..., 2]
                fy = w[..., 1] if by else a[..., 1]
                fx = w[..., 0] if bx else a[..., 0]
                v_all[..., c, :] = ((g * fz[..., None]) * fy[..., None]) * fx[..., None]
            keys, vals = k_all.reshape(-1), v_all.reshape(-1, 2)
    tab = np.zeros((L * T, 2), np.float32)
    np.add.at(tab, keys.astype(np.int64), vals)
    return tab


CASES = ["near_L16_T12", "smooth_L16_T12", "lin_L8_T14_r2_512"]


@pytest.mark.parametrize("name", CASES)
def test_serial_restatement_matches_reference(name):
    d = G.load("hashgrid")
    L, mn, mx, log2T, seed, interp = [int(v) for v in d[f"{name}:cfg"]]
    tab = serial_scatter(d["x01"], d[f"{name}:gy"], d[f"{name}:resolutions"], L, log2T, interp)
    ref = d[f"{name}:gtable"]
    np.testing.assert_allclose(tab, ref, rtol=0, atol=2e-5 * max(1.0, float(np.abs(ref).max())))


@pytest.mark.gpu
@pytest.mark.parametrize("name", CASES)
def test_deterministic_bwd_bit_exact_vs_serial(name):
    from adaptive_city_nerf_amd import ops
    d = G.load("hashgrid")
    L, mn, mx, log2T, seed, interp = [int(v) for v in d[f"{name}:cfg"]]
    x, gy = torch.from_numpy(d["x01"]).cuda(), torch.from_numpy(d[f"{name}:gy"]).cuda()
    got = ops.hashgrid_bwd(x, gy, d[f"{name}:resolutions"].tolist(), log2T, 2, interp, deterministic=True)
    np.testing.assert_array_equal(got.cpu().numpy(), serial_scatter(d["x01"], d[f"{name}:gy"],
                                                                     d[f"{name}:resolutions"], L, log2T, interp))


@pytest.mark.gpu
@pytest.mark.parametrize("interp", [1, 2])
def test_deterministic_bwd_full_table_reproducible(interp):
    """The reference configuration (L=16, T=2^20, 4095 finest) on 60k points concentrated along a few
    rays (long runs of equal rows at the coarse levels): bit-exact vs the serial scatter, identical
    over repeated runs; the float-atomic kernel agrees to fp32 rounding."""
    from adaptive_city_nerf_amd import ops
    from oracle import oracle as O
    res = O.level_resolutions(16, 16, 4096)
    g = torch.Generator().manual_seed(5)
    o = torch.rand(200, 1, 3, generator=g) * 0.8 + 0.1
    dd = torch.nn.functional.normalize(torch.randn(200, 1, 3, generator=g), dim=-1) * 0.08
    t = torch.linspace(0, 1, 300).view(1, -1, 1)
    x = (o + dd * t).reshape(-1, 3).clamp(1e-6, 1 - 1e-6).contiguous()
    gy = torch.randn(x.shape[0], 32, generator=g) * 1e-3
    ref = serial_scatter(x.numpy(), gy.numpy(), res, 16, 20, interp)
    a = ops.hashgrid_bwd(x.cuda(), gy.cuda(), res.tolist(), 20, 2, interp, deterministic=True)
    b = ops.hashgrid_bwd(x.cuda(), gy.cuda(), res.tolist(), 20, 2, interp, deterministic=True)
    np.testing.assert_array_equal(a.cpu().numpy(), ref)
    assert torch.equal(a, b)
    c = ops.hashgrid_bwd(x.cuda(), gy.cuda(), res.tolist(), 20, 2, interp, deterministic=False)
    np.testing.assert_allclose(c.cpu().numpy(), ref, rtol=0, atol=4e-6 * float(np.abs(ref).max()))


@pytest.mark.gpu
def test_torch_deterministic_flag_selects_sorted_backward():
    from adaptive_city_nerf_amd.encodings import HashGridEncoder
    enc = HashGridEncoder(levels=16, log2_hashmap_size=14, features_per_level=2, interpolation="Linear").cuda()
    x = torch.rand(5000, 3, device="cuda")
    gy = torch.randn(5000, 32, device="cuda")
    prev = torch.are_deterministic_algorithms_enabled()
    torch.use_deterministic_algorithms(True)
    try:
        grads = []
        for _ in range(2):
            enc.hash_table.grad = None
            (enc(x) * gy).sum().backward()
            grads.append(enc.hash_table.grad.clone())
    finally:
        torch.use_deterministic_algorithms(prev)
    assert torch.equal(grads[0], grads[1])
    ref = serial_scatter(x.cpu().numpy(), gy.cpu().numpy(), enc._res_host, 16, 14, 1)
    np.testing.assert_array_equal(grads[0].cpu().numpy(), ref)
