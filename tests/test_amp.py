"""use_amp: the training MLP in the reference's autocast(float16) arithmetic and GradScaler.

The reference trains with use_amp=True on GPU (configs/train.json:37; runtime_adapt.py:232-268): the MetaLinear
chain runs under torch.autocast(float16) and the update goes through torch.cuda.amp.GradScaler.  The _amp MLP
kernels (mlp_train.hip built with ACN_TRAIN_AMP=1) and optim.AmpScaler restate that:
  * against torch's own autocast chain on the same GPU (hipBLASLt fp16 GEMMs, the reference's arithmetic): the
    fp16 roundings agree up to the GEMMs' fp32 summation order -- a few fp16 ulps of drift through 6 layers;
  * against the fp32 chain (the parity oracle): the fp16 error itself, reported and bounded;
  * GradScaler: a finite step keeps / grows the scale on schedule, a non-finite gradient skips the update (no
    parameter, moment or step-count change; gradients cleared) and halves the scale."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

WNAMES = ("w0", "b0", "w1", "b1", "wsh", "bsh", "wg", "bg", "wc0", "bc0", "wc1", "bc1", "wc2", "bc2")


class _TruncExp(torch.autograd.Function):
    """models/trunc_exp.py: clamp at the dtype's exp limit (the scalar cast to the tensor's dtype), exp;
    backward grad * exp(xc) (no clamp mask)."""

    @staticmethod
    def forward(ctx, x):
        m = {torch.float16: 11.089866488}.get(x.dtype, 88.722839111)
        xc = x.clamp(-m, m)
        ctx.save_for_backward(xc)
        return torch.exp(xc)

    @staticmethod
    def backward(ctx, g):
        (xc,) = ctx.saved_tensors
        return g * torch.exp(xc)


def torch_chain(h0, sh, ws, amp):
    """The expert MLP of meta_ngp.py (density: trunk -> [geo | sigma] heads; color: [geo, SH] -> 64 -> 64 -> 3)
    with F.linear, optionally under torch.autocast(float16) as the reference's use_amp runs it."""
    w = dict(zip(WNAMES, ws))
    with torch.autocast("cuda", dtype=torch.float16, enabled=amp):
        a1 = F.relu(F.linear(h0, w["w0"], w["b0"]))
        a2 = F.relu(F.linear(a1, w["w1"], w["b1"]))
        sig = _TruncExp.apply(F.linear(a2, w["wsh"], w["bsh"]))
        geo = F.linear(a2, w["wg"], w["bg"])
        cin = torch.cat([geo, sh], -1)
        c1 = F.relu(F.linear(cin, w["wc0"], w["bc0"]))
        c2 = F.relu(F.linear(c1, w["wc1"], w["bc1"]))
        rgb = torch.sigmoid(F.linear(c2, w["wc2"], w["bc2"]))
        return torch.cat([rgb.float(), sig.float()], -1)


def _weights(seed, scale=0.4):
    from adaptive_city_nerf_amd import ops
    g = torch.Generator().manual_seed(seed)
    shapes = {"w0": (64, 32), "b0": (64,), "w1": (64, 64), "b1": (64,), "wsh": (1, 64), "bsh": (1,), "wg": (15, 64),
              "bg": (15,), "wc0": (64, 31), "bc0": (64,), "wc1": (64, 64), "bc1": (64,), "wc2": (3, 64), "bc2": (3,)}
    assert tuple(shapes[n] for n in WNAMES) == tuple(ops.MLP_DW_SHAPES)
    return [((torch.rand(shapes[n], generator=g) - 0.5) * scale).cuda() for n in WNAMES]


def _data(n, seed):
    g = torch.Generator(device="cuda").manual_seed(seed)
    h0 = (torch.rand(n, 32, device="cuda", generator=g) - 0.5) * 2
    sh = (torch.rand(n, 16, device="cuda", generator=g) - 0.5) * 2
    gout = torch.randn(n, 4, device="cuda", generator=g) * 1e-4   # an MSE gradient's size (1 / n_samples)
    return h0, sh, gout


def _ours(h0, sh, gout, ws, precision):
    from adaptive_city_nerf_amd import ops
    out, _ = ops.mlp_train_fwd(h0, sh, ws, save=False, precision=precision)
    grads, gh = ops.mlp_train_bwd_dw(h0, sh, out, gout, ws, want_h0=True, precision=precision)
    return out, [g.clone() for g in grads], gh


def _torch(h0, sh, gout, ws, amp):
    h = h0.clone().requires_grad_(True)
    wr = [w.clone().requires_grad_(True) for w in ws]
    out = torch_chain(h, sh, wr, amp)
    gr = torch.autograd.grad(out, [h] + wr, grad_outputs=gout)
    return out.detach(), list(gr[1:]), gr[0]


def _dev(a, b):
    a, b = a.double().cpu().numpy(), b.double().cpu().numpy()
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-30))


@pytest.mark.parametrize("n", [1, 777, 65536 + 5])
def test_amp_mlp_matches_torch_autocast(n):
    """Outputs, dL/dh0 and the 14 [dW | db] against torch.autocast(float16) on the same GPU, with the loss
    scale applied to the output gradient as GradScaler does (2^16)."""
    ws = _weights(3)
    h0, sh, gout = _data(n, n)
    S = 2.0 ** 16
    o_a, g_a, h_a = _ours(h0, sh, gout * S, ws, "amp")
    o_t, g_t, h_t = _torch(h0, sh, gout * S, ws, True)
    # every output of ours is an fp16 value, like autocast's
    assert torch.equal(o_a, o_a.half().float())
    assert torch.isfinite(o_a).all() and torch.isfinite(h_a).all()
    # rgb: most values bit-equal (the GEMM summation order moves a few roundings only); sigma: torch's half
    # exp on this stack rounds differently from expf-then-round, within an fp16 ulp or two
    same = float((o_a[:, :3] == o_t[:, :3]).float().mean())
    assert same >= 0.9, same
    assert _dev(o_a[:, :3], o_t[:, :3]) <= 4e-3
    sa, st_ = o_a[:, 3].double(), o_t[:, 3].double()
    assert float(((sa - st_).abs() / st_.abs().clamp_min(1e-30)).max()) <= 2.0 ** -9
    # gradients: both sides carry fp16 rounding through the chain; the same error scale as autocast's own
    _, g64, h64 = _torch(h0.double(), sh.double(), gout.double() * S, [w.double() for w in ws], False)
    assert _dev(h_a, h_t) <= max(0.25, 2 * _dev(h_t, h64)) and _dev(h_a, h64) <= 2 * _dev(h_t, h64) + 1e-3
    for name, a, b, r in zip(WNAMES, g_a, g_t, g64):
        assert torch.equal(a, a.half().float()), name       # [dW | db] rounded to fp16 once
        assert _dev(a, r) <= 2 * _dev(b, r) + 1e-3, (name, _dev(a, r), _dev(b, r))


def test_amp_mlp_error_against_fp32_oracle():
    """The fp16 arithmetic's own error, against the fp32 chain (float64 on the host): bounded and reported;
    the fp16x3 kernels on the same inputs stay ~1e-6 (the parity mode)."""
    ws = _weights(5)
    h0, sh, gout = _data(4096, 9)
    S = 2.0 ** 16
    o64, g64, h64 = _torch(h0.double(), sh.double(), gout.double() * S, [w.double() for w in ws], False)
    o_a, g_a, h_a = _ours(h0, sh, gout * S, ws, "amp")
    o_t, g_t, h_t = _torch(h0, sh, gout * S, ws, True)
    o_x, g_x, h_x = _ours(h0, sh, gout * S, ws, "fp16x3")
    rep = {"out": (_dev(o_a, o64), _dev(o_t, o64), _dev(o_x, o64)),
           "dh0": (_dev(h_a, h64), _dev(h_t, h64), _dev(h_x, h64))}
    for name, a, t, x, r in zip(WNAMES, g_a, g_t, g_x, g64):
        rep[name] = (_dev(a, r), _dev(t, r), _dev(x, r))
    print("AMPREPORT", {k: f"amp {v[0]:.2e} torch-autocast {v[1]:.2e} fp16x3 {v[2]:.2e}" for k, v in rep.items()})
    # the _amp kernels' error is the reference's own autocast error (max |dev| / max |ref| per tensor)
    assert all(v[0] <= 2 * v[1] + 1e-3 for v in rep.values()), rep
    assert max(v[2] for v in rep.values()) <= 5e-5


def test_amp_underflow_without_loss_scale():
    """What GradScaler exists for: unscaled MSE-sized gradients (1e-8) underflow fp16 in the backward, the
    loss-scaled ones do not (the kernels apply no hidden rescaling)."""
    ws = _weights(7)
    h0, sh, gout = _data(2048, 4)
    _, g1, _ = _ours(h0, sh, gout * 1e-4, ws, "amp")               # ~1e-8 output gradients
    _, gS, _ = _ours(h0, sh, gout * 1e-4 * 2.0 ** 16, ws, "amp")
    z1 = sum(int((g == 0).sum()) for g in g1)
    zS = sum(int((g == 0).sum()) for g in gS)
    assert z1 > zS


def _c5_step(amp, graph=False, clear=False):
    import goldens as G
    from types import SimpleNamespace
    from test_module_api import build_model, reference_state_dict
    from adaptive_city_nerf_amd import ops
    from adaptive_city_nerf_amd.optim import build_optimizer
    from adaptive_city_nerf_amd.routed_train import RoutedAdaptStep
    d = G.load("train_k8")
    P = SimpleNamespace(ray_samples=96, chunk_points=4_000_000, color_space="linear", optimizer="adam", lr=1e-4,
                        encoding_lr=0.01, sigma_lr=0.002, color_lr=0.002, bg_lr=0.001, weight_decay=0.0)
    was = ops.TRAIN_MLP_PRECISION
    ops.set_train_mlp_precision("amp" if amp else "fp16x3")
    try:
        m, _ = build_model("k8")
        m.load_state_dict(reference_state_dict(d, 8, "w:"))
        m = m.cuda().train()
        opt = build_optimizer(P, m)
        st = RoutedAdaptStep(P, m, int(d["train0:rays"].shape[0]), opt, grad_clip=1.0, graph=graph,
                             jitter="given", clear_in_adam=clear)
    finally:
        ops.set_train_mlp_precision(was)
    return d, m, st


def _run(st, d, i=0):
    return st(torch.from_numpy(d[f"train{i}:rays"]).cuda(), torch.from_numpy(d[f"train{i}:rgbs"]).cuda(),
              jitter_u=torch.from_numpy(d[f"train{i}:u"]).cuda())


def test_amp_c5_step_against_reference_fixture():
    """RoutedAdaptStep with use_amp: the step-0 loss and (unscaled) MLP gradients against the reference's fp32
    fixture within fp16 arithmetic's error; GradScaler state after a finite step: scale 2^16, tracker 1."""
    d, m, st = _c5_step(True)
    loss = float(_run(st, d))
    torch.cuda.synchronize()
    assert abs(loss - float(d["train0:loss"])) <= 2e-3 * abs(float(d["train0:loss"]))
    sd = st.amp.state_dict()
    assert sd["scale"] == 2.0 ** 16 and sd["_growth_tracker"] == 1 and not st.amp.found_inf()
    S = sd["scale"]
    worst = 0.0
    for n, p in m.named_parameters():
        key = f"train0:grad:{n}"
        if p.grad is None or key not in d or n.endswith("hash_table") or "bg_mlp" in n:
            continue
        ref = d[key].astype(np.float64)
        g = p.grad.double().cpu().numpy() / S
        worst = max(worst, float(np.linalg.norm(g - ref) / max(np.linalg.norm(ref), 1e-30)))
    assert worst <= 5e-2, worst


def test_amp_found_inf_skips_and_backs_off():
    """A loss scale large enough to overflow fp16 in the backward (2^40): the step is skipped -- parameters,
    Adam moments and step counters unchanged, gradients cleared -- and the scale halves; the next step at
    the halved scale (still overflowing) skips again, and a sane scale steps normally."""
    d, m, st = _c5_step(True, clear=True)
    before = {n: p.detach().clone() for n, p in m.named_parameters()}
    steps0 = st.adam.step_dev.clone()
    st.amp.scale_t.fill_(2.0 ** 40)
    _run(st, d)
    torch.cuda.synchronize()
    assert st.amp.found_inf()
    assert st.amp.get_scale() == 2.0 ** 39 and st.amp.state_dict()["_growth_tracker"] == 0
    assert torch.equal(st.adam.step_dev, steps0)
    for n, p in m.named_parameters():
        assert torch.equal(p.detach(), before[n]), n
    for g in st.gtables:      # the table gradients were cleared as the Adam pass clears them after an update
        assert int((g != 0).sum()) == 0
    if st.segmaps is not None:
        assert int(st.segmaps[:, 0].sum()) == 0       # no segment left marked "touched now"
    for r in st.adam.rows:
        assert torch.isfinite(r[2]).all() and torch.isfinite(r[3]).all()
    st.amp.scale_t.fill_(2.0 ** 16)
    _run(st, d, 1)
    torch.cuda.synchronize()
    assert not st.amp.found_inf()
    assert int((st.adam.step_dev - steps0).max()) == 1
    assert any(not torch.equal(p.detach(), before[n]) for n, p in m.named_parameters())


def test_amp_scale_growth_interval():
    """update(): the scale doubles after growth_interval consecutive finite steps (interval 2 here)."""
    d, m, st = _c5_step(True)
    st.amp.growth_interval = 2
    _run(st, d, 0)
    assert st.amp.get_scale() == 2.0 ** 16 and st.amp.state_dict()["_growth_tracker"] == 1
    _run(st, d, 1)
    assert st.amp.get_scale() == 2.0 ** 17 and st.amp.state_dict()["_growth_tracker"] == 0


def test_amp_c5_graph_replay_matches_eager():
    """The captured step replays the GradScaler update on the device: graph-replayed AMP steps track the eager
    ones (same batches, same jitter; the table scatter's float atomics allow last-bit differences) and end
    with the same scaler state (two growths at interval 2)."""
    d, m1, st1 = _c5_step(True, graph=False)
    d, m2, st2 = _c5_step(True, graph=True)
    st1.amp.growth_interval = st2.amp.growth_interval = 2
    for i in range(4):
        a, b = float(_run(st1, d, i % 3)), float(_run(st2, d, i % 3))
        assert abs(a - b) <= 1e-4 * abs(a), (i, a, b)
    torch.cuda.synchronize()
    assert st2.replays >= 1
    assert st1.amp.state_dict() == st2.amp.state_dict() and st1.amp.get_scale() == 2.0 ** 18   # 4 steps, interval 2


def test_amp_graphed_meta_step_matches_eager_gradscaler(monkeypatch):
    """Offline meta-training with use_amp (trainer.py:24 GradScaler, meta_core.py:123-136): the drop-in
    train_step replaying the task graphs + the outer graph with the GradScaler's device state, against the
    eager train_step driving torch's own GradScaler (scale / unscale_ / clip / step / update) with the same
    _amp kernels: the same updates to fp32 summation order and the same scaler state."""
    import contextlib
    import goldens as G
    from test_meta_gpu import _P, _compare_meta_runs, _model_and_tasks
    from adaptive_city_nerf_amd import meta_train as MT
    from adaptive_city_nerf_amd import ops
    from adaptive_city_nerf_amd.optim import build_optimizer
    d = G.load("meta_fomaml")
    P = _P("fomaml")
    P.use_amp = True
    was = ops.TRAIN_MLP_PRECISION
    ops.set_train_mlp_precision("amp")
    try:
        ma, tasks = _model_and_tasks(d)
        mb, _ = _model_and_tasks(d)
        oa, ob = build_optimizer(P, ma), build_optimizer(P, mb)
        sa, sb = torch.amp.GradScaler("cuda", growth_interval=2), torch.amp.GradScaler("cuda", growth_interval=2)
        monkeypatch.setattr(MT, "FAST_META_STEP", False)
        torch.manual_seed(7)
        with contextlib.redirect_stdout(None):
            for step in range(4):
                ra = MT.train_step(P, step, ma, oa, tasks, grad_scaler=sa)
        monkeypatch.setattr(MT, "FAST_META_STEP", True)
        torch.manual_seed(7)
        with contextlib.redirect_stdout(None):
            for step in range(4):
                rb = MT.train_step(P, step, mb, ob, tasks, grad_scaler=sb)
        g = ob._acn_meta_graph
        assert isinstance(g, MT.GraphedMetaStep) and g.amp is not None and g.replays == 3
        torch.cuda.synchronize()
        g.sync_state()
        assert sa.get_scale() == sb.get_scale() == 2.0 ** 18        # 4 finite steps at interval 2: two growths
        assert sa.state_dict()["_growth_tracker"] == sb.state_dict()["_growth_tracker"] == 0
        _compare_meta_runs(ma, oa, mb, ob, ra, rb, lambda n: 4)
    finally:
        ops.set_train_mlp_precision(was)


def test_expert_parallel_step_rejects_amp_without_loss_scale():
    """the expert-parallel step carries no loss scale, so it refuses the use_amp kernels."""
    from types import SimpleNamespace
    import goldens as G
    from test_module_api import build_model, reference_state_dict
    from adaptive_city_nerf_amd import ops
    from adaptive_city_nerf_amd._lib import AcnError
    from adaptive_city_nerf_amd.expert_parallel import ExpertParallelAdaptStep
    from adaptive_city_nerf_amd.optim import build_optimizer
    d = G.load("train_k8")
    P = SimpleNamespace(ray_samples=96, chunk_points=4_000_000, color_space="linear", optimizer="adam", lr=1e-4,
                        encoding_lr=0.01, sigma_lr=0.002, color_lr=0.002, bg_lr=0.001, weight_decay=0.0)
    m, _ = build_model("k8")
    m.load_state_dict(reference_state_dict(d, 8, "w:"))
    m = m.cuda().train()
    opt = build_optimizer(P, m)
    was = ops.TRAIN_MLP_PRECISION
    ops.set_train_mlp_precision("amp")
    try:
        with pytest.raises(AcnError, match="loss scale"):
            ExpertParallelAdaptStep(P, m, 1000, opt)
    finally:
        ops.set_train_mlp_precision(was)


def test_eager_adapt_step_under_amp_uses_a_grad_scaler():
    """the eager adapt_step (ragged batches, active_module updates) with the use_amp kernels runs
    under a GradScaler as the reference's runtime_adapt does (runtime_adapt.py:237-268): the loss scale reaches
    the fp16 backward (no underflow to all-zero tables) and the step equals the fp16x3 step within use_amp's
    tolerance; the scaler's scale is used and kept."""
    from types import SimpleNamespace
    import goldens as G
    from test_module_api import build_model, reference_state_dict
    from adaptive_city_nerf_amd import ops
    from adaptive_city_nerf_amd.optim import build_optimizer
    from adaptive_city_nerf_amd.train import adapt_step
    d = G.load("train_k8")
    P = SimpleNamespace(ray_samples=96, chunk_points=4_000_000, color_space="linear", optimizer="adam", lr=1e-4,
                        encoding_lr=0.01, sigma_lr=0.002, color_lr=0.002, bg_lr=0.001, weight_decay=0.0)
    rays = torch.from_numpy(d["train0:rays"]).cuda()
    rgbs = torch.from_numpy(d["train0:rgbs"]).cuda()
    u = torch.from_numpy(d["train0:u"]).cuda()
    res = {}
    was = ops.TRAIN_MLP_PRECISION
    for prec in ("fp16x3", "amp"):
        ops.set_train_mlp_precision(prec)
        try:
            m, _ = build_model("k8")
            m.load_state_dict(reference_state_dict(d, 8, "w:"))
            m = m.cuda().train()
            opt = build_optimizer(P, m)
            gs = torch.amp.GradScaler("cuda")
            loss = adapt_step(P, m, rays, rgbs, opt, active_module=2, grad_clip=1.0, grad_scaler=gs, jitter_u=u)
            g = m.submodules[2].xyz_encoder.hash_table.grad
            res[prec] = (float(loss), None if g is None else g.detach().clone(), gs.get_scale())
        finally:
            ops.set_train_mlp_precision(was)
    (l0, g0, _), (l1, g1, s1) = res["fp16x3"], res["amp"]
    assert abs(l1 - l0) <= 2e-3 * l0
    assert s1 == 2.0 ** 16                     # a finite first step keeps the initial scale
    assert g1 is not None and int((g1 != 0).sum()) > 0.9 * int((g0 != 0).sum())


def test_amp_scaler_wrap_state_dict_and_reset():
    """state_dict() of an AmpScaler wrapping a torch GradScaler (0-dim tracker); reset() restores a
    fresh scaler's state (one GradScaler per runtime_adapt call in the reference)."""
    from adaptive_city_nerf_amd.optim import AmpScaler
    gs = torch.amp.GradScaler("cuda", init_scale=1024.0)
    a = AmpScaler.wrap(gs, torch.device("cuda"))
    sd = a.state_dict()
    assert sd["scale"] == 1024.0 and sd["_growth_tracker"] == 0
    a.scale_t.fill_(8.0)
    a.tracker.fill_(3)
    assert a.state_dict()["_growth_tracker"] == 3 and gs.get_scale() == 8.0
    a.reset()
    assert a.get_scale() == 2.0 ** 16 and a.state_dict()["_growth_tracker"] == 0
