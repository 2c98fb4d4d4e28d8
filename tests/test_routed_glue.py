"""The fused glue of the routed adaptation step (VERDICT r04 "Next" 6) against the launches it replaces.

acn_routed_composite_mse_train runs the blend, background forward, compositing, linear-space MSE and their
backward down to the pair outputs in one launch; acn_grad_clip_slots runs the clip norm's partial sums, their
reduction and the clip coefficient in one launch.  Both keep the arithmetic of the separate kernels, so the
reference's K = 8 runtime_adapt steps (train_k8.npz batches, deterministic table backward) leave parameters,
both Adam moments, the clip norm and the per-step losses BITWISE equal with the fusions on and off -- full
batches and a ragged one (fewer rays than the step was built for), fp16x3 and use_amp.  Reference:
pipelines/online_stage/runtime_adapt.py:286-309, nerfs/ray_rendering.py:137-165, nerfs/losses.py:10-32."""
from types import SimpleNamespace

import pytest
import torch

import goldens as G
from test_train import P

pytestmark = pytest.mark.gpu


def _run(monkeypatch, composite, clip, precision="fp16x3", steps=4, S=96, n_rays=1000):
    from test_module_api import build_model, reference_state_dict
    from adaptive_city_nerf_amd import ops
    from adaptive_city_nerf_amd import optim as O
    from adaptive_city_nerf_amd import routed_train as RT
    monkeypatch.setattr(RT, "FUSED_COMPOSITE", composite)
    monkeypatch.setattr(O, "FUSED_CLIP", clip)
    d = G.load("train_k8")
    Pk = SimpleNamespace(**{**vars(P), "ray_samples": S, "chunk_points": 4_000_000})
    g = torch.Generator().manual_seed(5)
    batches = [(torch.from_numpy(d[f"train{s}:rays"][:n_rays]).cuda(), torch.from_numpy(d[f"train{s}:rgbs"][:n_rays]).cuda(),
                torch.from_numpy(d[f"train{s}:u"][:n_rays]).cuda() if S == 96 else
                torch.rand(n_rays, S, generator=g).cuda()) for s in range(3)]
    was = ops.TRAIN_MLP_PRECISION
    ops.set_train_mlp_precision(precision)
    torch.use_deterministic_algorithms(True)
    try:
        m, _ = build_model("k8")
        m.load_state_dict(reference_state_dict(d, 8, "w:"))
        m = m.cuda().train()
        opt = O.build_optimizer(Pk, m)
        st = RT.RoutedAdaptStep(Pk, m, n_rays, opt, grad_clip=1.0, graph=False, jitter="given")
        losses, norms = [], []
        for i in range(steps):
            r, c, u = batches[i % 3]
            if i == steps - 1:          # a ragged batch through the same buffers
                k = max(1, (613 * n_rays) // 1000)
                r, c, u = r[:k], c[:k], u[:k]
            losses.append(float(st(r, c, jitter_u=u)))
            norms.append(st.last_norm.detach().cpu().clone())
        torch.cuda.synchronize()
        st.sync_state()
        params = {n: (p.detach().clone(), opt.state[p]["exp_avg"].clone(), opt.state[p]["exp_avg_sq"].clone())
                  for n, p in m.named_parameters() if p in opt.state}
        return losses, norms, params
    finally:
        torch.use_deterministic_algorithms(False)
        ops.set_train_mlp_precision(was)


@pytest.mark.parametrize("precision", ["fp16x3", "amp"])
def test_fused_composite_and_clip_bitwise_equal_separate_launches(monkeypatch, precision):
    fused = _run(monkeypatch, True, True, precision)
    plain = _run(monkeypatch, False, False, precision)
    assert fused[0] == plain[0], (fused[0], plain[0])
    for a, b in zip(fused[1], plain[1]):
        assert torch.equal(a, b), (a, b)
    assert fused[2].keys() == plain[2].keys()
    for n in fused[2]:
        for a, b in zip(fused[2][n], plain[2][n]):
            assert torch.equal(a, b), n
    # and each fusion on its own
    mixed = _run(monkeypatch, True, False, precision, steps=2)
    ref2 = _run(monkeypatch, False, True, precision, steps=2)
    assert mixed[0] == ref2[0]
    for n in mixed[2]:
        for a, b in zip(mixed[2][n], ref2[2][n]):
            assert torch.equal(a, b), n


def test_fused_composite_bitwise_equal_separate_launches_long_rays(monkeypatch):
    """S = 200 (> 128): the fused kernel's blend backward reloads each sample's pair slots instead of keeping them
    in registers; two steps and a ragged one, bitwise equal to the separate launches."""
    fused = _run(monkeypatch, True, True, steps=3, S=200)
    plain = _run(monkeypatch, False, False, steps=3, S=200)
    assert fused[0] == plain[0], (fused[0], plain[0])
    for n in fused[2]:
        for a, b in zip(fused[2][n], plain[2][n]):
            assert torch.equal(a, b), n


@pytest.mark.parametrize("n_rays,S", [(5, 2), (7, 33), (3, 129)])
def test_fused_composite_bitwise_equal_separate_launches_small_sizes(monkeypatch, n_rays, S):
    """Edge sizes of the fused launch: a ray count that is not a multiple of the workgroup's 4 waves, the minimum
    S = 2, a partial last 32-sample tile, and S just past 128 (the reload path); two steps, bitwise."""
    fused = _run(monkeypatch, True, True, steps=2, S=S, n_rays=n_rays)
    plain = _run(monkeypatch, False, False, steps=2, S=S, n_rays=n_rays)
    assert fused[0] == plain[0], (fused[0], plain[0])
    for n in fused[2]:
        for a, b in zip(fused[2][n], plain[2][n]):
            assert torch.equal(a, b), n
