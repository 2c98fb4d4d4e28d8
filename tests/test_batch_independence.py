"""Ray independence of the routed render (VERDICT r03 "what's weak" 4).

The reference renders every ray on its own (nerfs/ray_rendering.py:290-345: each ray's t-values, field
queries and compositing touch no other ray), so a ray's rgb / depth / acc / weights must not depend on
which other rays share its batch.  render_slots_kernel (K > 2) keeps the two experts its workgroup
round needs most in LDS and reads the others from L2: that choice depends on the neighbouring rays,
and round 3 found a ray whose arithmetic changed with it (colour layer 0 folded on one path, unfolded
on the other).  These tests pin bitwise equality per ray across batch compositions that move every
ray through different workgroup rounds and slot assignments: the fixture order, a random
permutation, the reverse, a ragged subset, a 5x replicated shuffled batch and 16-ray batches (one
workgroup round each), for the K=4 and K=8 fixtures, eval and training jitter, with and without
early termination."""
import numpy as np
import pytest
import torch

import goldens as G
from oracle import oracle as O

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _t(a):
    return torch.from_numpy(np.ascontiguousarray(a)).to(DEV)


def _setup(tag, prefix, scale):
    from adaptive_city_nerf_amd import ops
    d = G.load(f"render_{tag}")
    mask = G.MASK[tag]
    sc = G.scene()["masks"][mask]
    K = len(sc["centroids"])
    res = O.level_resolutions(16, 16, 4096)
    specs = []
    for k in range(K):
        w = G.expert_weights(d, k, prefix)
        tab = _t(G.table(int(d["table_seeds"][k]), float(d["table_scale"]) if scale is None else scale))
        mlp = {key: _t(v) for key, v in w.items() if key in ops.MLP_SHAPES}
        specs.append(ops.ExpertSpec(tab, res.tolist(), 20, 1, sc["mins"][k],
                                    d[f"w:submodules.{k}.aabb_extent"].tolist(), mlp))
    routing = ops.make_routing(torch.tensor(sc["centroids"]), K, True, float(d["bm"]))
    bgw = {k[len("bg_mlp."):]: _t(v) for k, v in G.bg_weights(d, prefix).items()}
    bg, keep = ops.make_background("mlp", mlp=bgw)
    return d, specs, routing, (bg, keep)


def _render(rays, jit, specs, routing, bg, tau, S):
    from adaptive_city_nerf_amd import ops
    return ops.render_stratified(rays, S, specs, routing, None, bg[0], tau=tau, jitter=jit)


def _same(a, b):
    return np.array_equal(a.cpu().numpy(), b.cpu().numpy(), equal_nan=True)


@pytest.mark.parametrize("tag,prefix,scale", [("k4", "w:", None), ("k4", "hiw:", None), ("k8", "w:", None),
                                              ("k8", "hiw:", None), ("k8", "w:", 1e-3)])
@pytest.mark.parametrize("jitter", [False, True])
@pytest.mark.parametrize("tau", [0.0, 1e-5])
def test_routed_render_bitwise_batch_independent(tag, prefix, scale, jitter, tau):
    d, specs, routing, bg = _setup(tag, prefix, scale)
    S = 64
    rays = _t(d["render:rays"])
    n = rays.shape[0]
    g = torch.Generator(device=DEV).manual_seed(17)
    jit = torch.rand(n, S, device=DEV, generator=g) if jitter else None
    with torch.no_grad():
        ref = _render(rays, jit, specs, routing, bg, tau, S)
        perm = torch.randperm(n, device=DEV, generator=g)
        rep = torch.cat([torch.randperm(n, device=DEV, generator=g) for _ in range(5)])
        batches = {
            "permutation": perm,
            "reverse": torch.arange(n - 1, -1, -1, device=DEV),
            "ragged_subset": perm[: 777 if n > 777 else n // 2 + 1],
            "replicated_5x": rep,
        }
        for name, idx in batches.items():
            out = _render(rays[idx].contiguous(), None if jit is None else jit[idx].contiguous(), specs, routing,
                          bg, tau, S)
            for o, r, what in zip(out, ref, ("rgb", "depth", "weights", "acc")):
                assert _same(o, r[idx]), f"{tag} {prefix} {name}: {what} differs from the full-batch render"
        # one workgroup round per call (16 rays = the slots kernel's 8 waves x 2 rounds at most)
        for lo in range(0, min(n, 160), 16):
            idx = perm[lo: lo + 16]
            out = _render(rays[idx].contiguous(), None if jit is None else jit[idx].contiguous(), specs, routing,
                          bg, tau, S)
            for o, r, what in zip(out, ref, ("rgb", "depth", "weights", "acc")):
                assert _same(o, r[idx]), f"{tag} {prefix} 16-ray batch at {lo}: {what} differs"


@pytest.mark.parametrize("n,dup", [(1, 4), (63, 4), (777, 4), (4096, 4), (8192, 4), (4096, 4096), (5000, 40)])
def test_ray_order_stable_and_reproducible(n, dup):
    """ray_order_kernel (acn_ray_order) sorts a batch by direction cell with a stable sort: the result is
    a permutation, identical on every call, and rays with identical directions (one cell) keep their
    index order.  dup = rays per distinct direction on average: 4 (the counting sort's per-cell ranks),
    4096 (every ray in one cell: the radix-pass fallback) and 40 (cells near the fallback threshold)."""
    from adaptive_city_nerf_amd import _lib, ops
    d = G.load("render_k1")
    base = d["render:rays"]
    rng = np.random.default_rng(n)
    # groups of duplicated rays: each distinct direction appears at several scattered indices
    src = rng.integers(0, base.shape[0], max(1, n // dup))
    rays = base[src[rng.integers(0, src.shape[0], n)]].copy()
    if n > 8:
        rays[5, 3:6] = np.nan      # invalid directions go to the last cell
        rays[6, 3:6] = 0.0
    r = _t(rays)
    outs = []
    for _ in range(3):
        o = torch.empty(n, dtype=torch.int32, device=DEV)
        ops.check(_lib.lib().acn_ray_order(ops.ptr(r), n, ops.ptr(o), ops.stream_of(r)), "acn_ray_order")
        outs.append(o.cpu().numpy())
    assert np.array_equal(np.sort(outs[0]), np.arange(n))
    assert all(np.array_equal(outs[0], o) for o in outs[1:])
    pos = np.empty(n, np.int64)
    pos[outs[0]] = np.arange(n)
    key = [tuple(x) for x in rays[:, 3:6].view(np.uint32)]
    groups = {}
    for i, k in enumerate(key):
        groups.setdefault(k, []).append(i)
    for idx in groups.values():      # idx ascending: their visiting positions must ascend too
        assert np.all(np.diff(pos[idx]) > 0), "rays of one cell are not visited in index order"
