"""hipGraph replay of the online-adaptation step (train.GraphedAdaptStep + FusedAdam's device step
table): the replayed updates equal eager adapt_step updates on the same batches.  The hash-grid
backward accumulates with float atomics (order-dependent in the last bits), so parameters are compared
within 1e-5 relative / 1e-7 absolute after several steps, as two eager runs differ."""
import numpy as np
import pytest
import torch

import goldens as G

pytestmark = pytest.mark.gpu


def _setup(seed=0):
    from test_module_api import build_model, reference_state_dict
    from test_train import P
    from adaptive_city_nerf_amd.optim import build_optimizer
    d = G.load("train_k4")
    m, _ = build_model("k4")
    m.load_state_dict(reference_state_dict(d, len(m.submodules), "w:"))
    m = m.cuda().train()
    return P, m, build_optimizer(P, m), d


def _batches(d, n, S=96):
    g = torch.Generator(device="cuda").manual_seed(5)
    rays = torch.from_numpy(d["train0:rays"]).cuda()
    out = []
    for _ in range(n):
        idx = torch.randint(0, rays.shape[0], (rays.shape[0],), device="cuda", generator=g)
        out.append((rays[idx].contiguous(), torch.rand(rays.shape[0], 3, device="cuda", generator=g),
                    torch.rand(rays.shape[0], S, device="cuda", generator=g)))
    return out


@pytest.mark.parametrize("active_module", [0, 2])
def test_graphed_adapt_step_matches_eager(active_module):
    from adaptive_city_nerf_amd.train import GraphedAdaptStep, adapt_step
    P, ma, oa, d = _setup()
    _, mb, ob, _ = _setup()
    batches = _batches(d, 6, S=P.ray_samples)
    # eager: warmup twice on batch 0, then batches 1..5
    seq = [batches[0], batches[0]] + batches[1:]
    for rays, rgbs, u in seq:
        la = adapt_step(P, ma, rays, rgbs, oa, active_module=active_module, grad_clip=1.0, jitter_u=u)
    g = GraphedAdaptStep(P, mb, batches[0][0], batches[0][1], ob, active_module=active_module, grad_clip=1.0,
                         warmup=2, jitter_u=batches[0][2])
    for rays, rgbs, u in batches[1:]:
        lb = g(rays, rgbs, jitter_u=u)
    torch.cuda.synchronize()
    g.sync_state()
    assert abs(float(la) - float(lb)) <= 1e-5 * abs(float(la)) + 1e-8
    for (na, pa), (nb, pb) in zip(ma.named_parameters(), mb.named_parameters()):
        a, b = pa.detach().cpu().numpy(), pb.detach().cpu().numpy()
        if na.endswith("hash_table"):
            # the table gradient is a float-atomic scatter-add: rows whose 7-step gradient sits at the
            # summation-order noise level get Adam steps (~lr / sqrt(v)-normalised) that depend on that
            # noise, in two eager runs as much as here; a few per million rows, bounded by 1e-4
            bad = np.abs(a - b) > 1e-5 * np.abs(a) + 1e-7
            assert bad.mean() <= 1e-5 and np.abs(a - b).max() <= 1e-4, (na, int(bad.sum()), np.abs(a - b).max())
        else:
            # the MLP sees the noise through the table after the first update: a weight whose gradient
            # sits near zero gets Adam steps (~lr sign(g)) that differ between runs; allow 1% of such
            # elements, each within 1e-3 of the sigma/colour lr (0.002) -- seen: 7 of 2048, 5.5e-7
            bad = np.abs(a - b) > 1e-5 * np.abs(a) + 1e-7
            assert bad.mean() <= 1e-2 and np.abs(a - b).max() <= 2e-6, (na, int(bad.sum()), np.abs(a - b).max())
    for pa, pb in zip(ma.parameters(), mb.parameters()):
        sa, sb = oa.state.get(pa, {}), ob.state.get(pb, {})
        assert ("step" in sa) == ("step" in sb)
        if "step" in sa:
            assert float(sa["step"]) == float(sb["step"]) == 7.0
            np.testing.assert_allclose(sb["exp_avg_sq"].cpu().numpy(), sa["exp_avg_sq"].cpu().numpy(), rtol=1e-4,
                                       atol=1e-12)


def test_graphed_adapt_step_with_device_rng_trains():
    from adaptive_city_nerf_amd.train import GraphedAdaptStep
    P, m, opt, d = _setup()
    batches = _batches(d, 4, S=P.ray_samples)
    before = [p.detach().clone() for p in m.parameters()]
    with pytest.raises(ValueError):
        GraphedAdaptStep(P, m, batches[0][0], batches[0][1], opt, grad_clip=1.0, warmup=1)
    g = GraphedAdaptStep(P, m, batches[0][0], batches[0][1], opt, active_module=3, grad_clip=1.0, warmup=1)
    losses = [float(g(r, c)) for r, c, _ in batches[1:]]
    torch.cuda.synchronize()
    assert all(np.isfinite(losses)) and g.replays == 3
    assert any(not torch.equal(a, b) for a, b in zip(before, m.parameters()))
