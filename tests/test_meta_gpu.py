"""GPU parity of the offline meta-training loop (adaptive_city_nerf_amd.meta_train, SURVEY §8(f)
rank 2) against the reference's own step (tests/golden/meta_*.npz): FOMAML and second-order MAML
train_step, the MAML inner loop alone, and the Reptile update rule, with the reference's recorded
training jitter replayed in call order."""
import contextlib
from types import SimpleNamespace

import numpy as np
import pytest
import torch

import goldens as G
from test_module_api import build_model, reference_state_dict

pytestmark = pytest.mark.gpu
LRS = {"encoding": 0.01, "sigma": 0.002, "color": 0.002, "background": 0.001}


def _P(algo):
    return SimpleNamespace(algo=algo, ray_samples=16, chunk_points=1 << 20, color_space="linear", optimizer="adam",
                           lr=1e-4, encoding_lr=0.01, sigma_lr=0.002, color_lr=0.002, bg_lr=0.001, weight_decay=0.0,
                           inner_lr=0.05, inner_iter=2, fim=False, use_amp=False, grad_clip=1.0, seed=0,
                           mixed_precision=False, print_step=10 ** 9)


@contextlib.contextmanager
def replay_jitter(us):
    """torch.rand_like of the (N, 16) training jitter returns the recorded draws in order."""
    real = torch.rand_like
    it = iter(us)

    def fake(t, *a, **k):
        if t.dim() == 2 and t.shape[1] == 16:
            return next(it).to(t.device, t.dtype).clone()
        return real(t, *a, **k)
    torch.rand_like = fake
    try:
        yield it
    finally:
        torch.rand_like = real


def _model_and_tasks(d):
    m, _ = build_model("k4")
    m.load_state_dict(reference_state_dict(d, 4))
    m = m.cuda().train()
    tasks = {cid: [{part: {"rays": torch.from_numpy(d[f"task{cid}:{part}:rays"]).cuda(),
                           "rgbs": torch.from_numpy(d[f"task{cid}:{part}:rgbs"]).cuda()}
                    for part in ("support", "query")}] for cid in (0, 2)}
    return m, tasks


def _close_frac(a, b, atol, rtol):
    a = np.asarray(a, np.float64); b = np.asarray(b, np.float64)
    return float(np.mean(np.abs(a - b) <= atol + rtol * np.abs(b)))


def _group(name):
    return "encoding" if name.endswith("hash_table") else "background" if name.startswith("bg_mlp") else \
        "color" if ".color_mlp." in name else "sigma"


def test_maml_inner_loop_matches_reference():
    from adaptive_city_nerf_amd import meta_train as MT
    d = G.load("meta_maml")
    m, tasks = _model_and_tasks(d)
    with replay_jitter(torch.from_numpy(d["u"])):
        fast, losses = MT.task_adapt(_P("maml"), m, tasks[0][0]["support"], 0.05, 2, active_module=0)
    np.testing.assert_allclose([float(x) for x in losses], d["adapt_inner_losses"], rtol=1e-5)
    for n, v in fast.items():
        ref = d["adapt_fast:" + n]
        np.testing.assert_allclose(v.detach().cpu().numpy(), ref, rtol=0, atol=1e-5 * max(1.0, np.abs(ref).max()),
                                   err_msg=n)


@pytest.mark.parametrize("algo", ["fomaml", "maml", "reptile"])
def test_train_step_matches_reference(algo):
    from adaptive_city_nerf_amd import meta_train as MT
    from adaptive_city_nerf_amd.optim import build_optimizer
    d = G.load(f"meta_{algo}")
    m, tasks = _model_and_tasks(d)
    P = _P(algo)
    opt = build_optimizer(P, m)
    us = torch.from_numpy(d["u"])
    if algo == "maml":
        us = us[2:]  # the fixture ran the inner loop alone first
    elif algo == "reptile":  # the fixture pinned the update rule without the query renders train_step adds
        q = torch.rand_like(us[0])
        us = torch.stack([us[0], us[1], q, us[2], us[3], q])
    with replay_jitter(us):
        MT.train_step(P, 1, m, opt, tasks)
    rows = torch.from_numpy(d["rows"]).cuda()
    for name, p in m.named_parameters():
        lr = LRS[_group(name)]
        if name.endswith("hash_table"):
            k = int(name.split(".")[1])
            got, ref = p.detach()[rows[k]].cpu().numpy(), d[f"after_table_rows:{k}"]
            if algo != "reptile" and f"grad_table_rows:{k}" in d:
                g = p.grad[rows[k]].cpu().numpy()
                gr = d[f"grad_table_rows:{k}"]
                np.testing.assert_allclose(g, gr, rtol=1e-3, atol=1e-4 * max(1e-12, np.abs(gr).max()), err_msg=name)
        else:
            got, ref = p.detach().cpu().numpy(), d["after:" + name]
            if algo != "reptile" and "grad:" + name in d:
                gr = d["grad:" + name]
                np.testing.assert_allclose(p.grad.cpu().numpy(), gr, rtol=0, atol=2e-4 * max(1e-12, np.abs(gr).max()),
                                           err_msg=name)
        # Adam's first step moves a parameter by ~lr * sign(g): a few near-zero gradients may flip
        assert _close_frac(got, ref, 1e-3 * lr, 1e-6) >= 0.998, name


def _compare_meta_runs(ma, oa, mb, ob, ra, rb, steps_expected):
    assert rb["loss_out"] == pytest.approx(ra["loss_out"], rel=1e-4)
    for (na, pa), (nb, pb) in zip(ma.named_parameters(), mb.named_parameters()):
        lr = LRS[_group(na)]
        assert _close_frac(pb.detach().cpu().numpy(), pa.detach().cpu().numpy(), 1e-3 * lr, 1e-5) >= 0.99, na
    for (na, pa), pb in zip(ma.named_parameters(), mb.parameters()):
        sa, sb = oa.state.get(pa, {}), ob.state.get(pb, {})
        assert ("step" in sa) == ("step" in sb), na
        if "step" in sa:
            assert float(sa["step"]) == float(sb["step"]) == float(steps_expected(na)), na


@pytest.mark.parametrize("algo", ["fomaml"])
@pytest.mark.parametrize("how", ["object", "drop_in"])
def test_graphed_meta_step_matches_eager(algo, how, monkeypatch):
    """GraphedMetaStep (per-region task graphs + outer slotted clip/Adam graph, jitter drawn inside the
    graphs) -- built explicitly, or reached through the drop-in train_step (first call eager, then capture
    + replay) -- against the eager train_step from the same RNG state: the same updates to fp32 order."""
    from adaptive_city_nerf_amd import meta_train as MT
    from adaptive_city_nerf_amd.optim import build_optimizer
    d = G.load(f"meta_{algo}")
    P = _P(algo)
    ma, tasks = _model_and_tasks(d)
    mb, _ = _model_and_tasks(d)
    oa, ob = build_optimizer(P, ma), build_optimizer(P, mb)
    monkeypatch.setattr(MT, "FAST_META_STEP", False)
    torch.manual_seed(7)
    with contextlib.redirect_stdout(None):
        for step in range(3):
            ra = MT.train_step(P, step, ma, oa, tasks)
    monkeypatch.setattr(MT, "FAST_META_STEP", True)
    torch.manual_seed(7)
    if how == "object":
        g = MT.GraphedMetaStep(P, mb, ob, tasks, warmup=1)
        for step in (1, 2):
            rb = g(step, tasks)
    else:
        with contextlib.redirect_stdout(None):
            for step in range(3):
                rb = MT.train_step(P, step, mb, ob, tasks)
        g = ob._acn_meta_graph
        assert isinstance(g, MT.GraphedMetaStep) and g.replays == 2 and g.eager_steps == 0
    torch.cuda.synchronize()
    g.sync_state()
    _compare_meta_runs(ma, oa, mb, ob, ra, rb, lambda n: 3)


def test_graphed_meta_step_region_without_tasks(monkeypatch):
    """a region with no task this step gets no gradient, so torch's Adam skips its expert (no
    moment decay, no step increment); the graphed step's slotted outer update does the same, and a step
    whose task shapes the graphs do not cover runs eagerly with the state carried over."""
    from adaptive_city_nerf_amd import meta_train as MT
    from adaptive_city_nerf_amd.optim import build_optimizer
    d = G.load("meta_fomaml")
    P = _P("fomaml")
    ma, tasks = _model_and_tasks(d)
    mb, _ = _model_and_tasks(d)
    oa, ob = build_optimizer(P, ma), build_optimizer(P, mb)
    cids = sorted(tasks)
    drop = cids[-1]
    partial = {c: (tasks[c] if c != drop else []) for c in cids}
    def _short(t):   # same region, fewer support rays: not covered by the captured shapes
        sup, qry = (t.support, t.query) if hasattr(t, "support") else (t["support"], t["query"])
        n = sup["rays"].shape[0] // 2
        return {"support": {k: v[:n] for k, v in sup.items()}, "query": qry}
    odd = {c: [_short(t) for t in tasks[c]] for c in cids}
    seq = [tasks, partial, tasks, odd, partial, tasks]
    results = []
    for fast, m, o in ((False, ma, oa), (True, mb, ob)):
        monkeypatch.setattr(MT, "FAST_META_STEP", fast)
        torch.manual_seed(11)
        with contextlib.redirect_stdout(None):
            for step, td in enumerate(seq):
                r = MT.train_step(P, step, m, o, td)
        results.append(r)
    g = ob._acn_meta_graph
    assert isinstance(g, MT.GraphedMetaStep) and g.eager_steps == 1 and g.replays == 4
    g.sync_state()
    n_drop = sum(1 for td in seq if td[drop])
    _compare_meta_runs(ma, oa, mb, ob, results[0], results[1],
                       lambda n: n_drop if n.startswith(f"submodules.{drop}.") else len(seq))


def test_graphed_meta_step_refuses_second_order():
    from adaptive_city_nerf_amd import meta_train as MT
    from adaptive_city_nerf_amd.optim import build_optimizer
    d = G.load("meta_maml")
    m, tasks = _model_and_tasks(d)
    with pytest.raises(ValueError):
        MT.GraphedMetaStep(_P("maml"), m, build_optimizer(_P("maml"), m), tasks)


def test_drop_in_train_step_state_dict_current_without_sync(monkeypatch):
    """the drop-in train_step leaves optimizer.state current after every replayed step, so the
    reference's checkpoint (optimizer.state_dict(), utils.py:290) is right without an explicit sync: step
    counts equal the eager run's, and an expert whose region first gets a task after the graphs were built
    (its state was pending inside the graph) appears with its real count."""
    from adaptive_city_nerf_amd import meta_train as MT
    from adaptive_city_nerf_amd.optim import build_optimizer
    d = G.load("meta_fomaml")
    P = _P("fomaml")
    ma, tasks = _model_and_tasks(d)
    mb, _ = _model_and_tasks(d)
    oa, ob = build_optimizer(P, ma), build_optimizer(P, mb)
    cids = sorted(tasks)
    drop = cids[-1]
    partial = {c: (tasks[c] if c != drop else []) for c in cids}
    seq = [partial, partial, tasks, tasks, partial]
    results = []
    for fast, m, o in ((False, ma, oa), (True, mb, ob)):
        monkeypatch.setattr(MT, "FAST_META_STEP", fast)
        torch.manual_seed(5)
        with contextlib.redirect_stdout(None):
            for step, td in enumerate(seq):
                r = MT.train_step(P, step, m, o, td)
        results.append(r)
    g = ob._acn_meta_graph
    # call 0 eager, call 1 captures and replays, call 2 captures the new region's graph (_covers) and replays
    assert isinstance(g, MT.GraphedMetaStep) and g.replays == 4 and g.eager_steps == 0
    sa, sb = oa.state_dict()["state"], ob.state_dict()["state"]
    assert sorted(sa) == sorted(sb)
    for i in sa:
        assert float(sa[i]["step"]) == float(sb[i]["step"]), i
    _compare_meta_runs(ma, oa, mb, ob, results[0], results[1],
                       lambda n: 2 if n.startswith(f"submodules.{drop}.") else len(seq))
