"""One expert per GPU (adaptive_city_nerf_amd/expert_parallel.py): the all-to-all of
per-sample records to the experts' owners and back, for rendering and for the runtime_adapt update of
the routed 8-expert container (BASELINE C5).

CPU: world size 2 over gloo; every rank holds a contiguous shard of the reference fixture's rays and
owns 4 of the 8 experts.  The compute is the CPU restatement (oracle/train_ref.py, pinned to the
reference's own train_k8 fixture) behind the backend interface, so what is checked here is the data
movement: the distributed render equals the single-process render and the distributed update equals
the reference's update (loss, clip norm, owned experts' gradients and parameters, the all-reduced
background head).  GPU: the HIP backend at world size 1 (the same code path, exchanges as copies)
against the fused render and the fixture.
"""
import os
import socket
from types import SimpleNamespace

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import goldens as G
from adaptive_city_nerf_amd.expert_parallel import (PairSet, adapt_step_expert_parallel, expert_owner,
                                                    render_rays_expert_parallel)
from oracle import oracle as O
from oracle import train_ref as TR

S = 96
LRS = {"encoding": 0.01, "sigma": 0.002, "color": 0.002, "background": 0.001}
P = SimpleNamespace(ray_samples=S, color_space="linear")


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def ref_container(d):
    sc = G.scene()["masks"][G.MASK["k8"]]
    K = len(sc["centroids"])
    state = {k[2:]: torch.from_numpy(v.copy()) for k, v in d.items() if k.startswith("w:")}
    for k in range(K):
        state[f"submodules.{k}.xyz_encoder.hash_table"] = torch.from_numpy(
            G.table(int(d["table_seeds"][k]), float(d["table_scale"])).copy())
    exts = [d[f"w:submodules.{k}.aabb_extent"] for k in range(K)]
    return TR.RefContainer(state, K, O.level_resolutions(16, 16, 4096), 20, sc["centroids"], float(d["bm"]), sc["mins"],
                           exts)


class RefBackend:
    """The backend interface on the CPU restatement (torch CPU autograd)."""

    def __init__(self, m):
        self.m = m

    def pairs(self, rays, S, u):
        o, dd = rays[:, :3], rays[:, 3:6]
        near, far = rays[:, 6], rays[:, 7]
        t_lin = torch.linspace(0.0, 1.0, S).unsqueeze(0)
        t = near.unsqueeze(1) * (1.0 - t_lin) + far.unsqueeze(1) * t_lin
        mids = 0.5 * (t[:, :-1] + t[:, 1:])
        t = torch.cat([t[:, :1], mids], 1) + (torch.cat([mids, t[:, -1:]], 1) - torch.cat([t[:, :1], mids], 1)) * u
        pts = (o.unsqueeze(1) + dd.unsqueeze(1) * t.unsqueeze(-1)).reshape(-1, 3)
        dirs = dd.unsqueeze(1).expand(-1, S, -1).reshape(-1, 3)
        x = torch.cat([pts, dirs], 1)
        with torch.no_grad():
            dist_ = torch.cdist(x[:, 1:3], self.m.cent[:, 1:3]).clamp_min(1e-6)
            invd = (1.0 / dist_) * (dist_ <= self.m.bm * dist_.min(1, keepdim=True).values)
            w = invd / invd.sum(1, keepdim=True).clamp_min(1e-6)
        K = self.m.K
        pmap = torch.full((x.shape[0], K), -1, dtype=torch.int64)
        pidx, pw, pk, counts, off = [], [], [], [], 0
        for k in range(K):
            sel = (w[:, k] > 0).nonzero(as_tuple=False).squeeze(1)
            pidx.append(sel); pw.append(w[sel, k]); pk.append(torch.full_like(sel, k)); counts.append(sel.numel())
            pmap[sel, k] = torch.arange(off, off + sel.numel())
            off += sel.numel()
        pidx = torch.cat(pidx)
        return PairSet(t, counts, pidx, torch.cat(pw), x[pidx], pmap, torch.cat(pk))

    def expert(self, k, xd):
        return self.m.expert(k, xd)

    def blend(self, y, ps):
        out = y.new_zeros(ps.pmap.shape[0], 4)
        off = 0
        for c in ps.counts:
            sl = slice(off, off + c)
            if c:
                out = out.index_add(0, ps.pidx[sl], y[sl] * ps.pw[sl].unsqueeze(1))
            off += c
        return out

    def composite(self, rs, t, rays):
        rgb = rs[..., :3].clamp(0.0, 1.0)
        sigma = rs[..., 3].clamp_min(0.0)
        dists = (t[:, 1:] - t[:, :-1]).clamp_min(1e-4)
        dists = torch.cat([dists, dists[:, -1:]], 1)
        alpha = (1.0 - torch.exp(-sigma * dists)).clamp(0.0, 1.0 - 1e-7)
        T = torch.cumprod(torch.cat([torch.ones_like(alpha[:, :1]), 1.0 - alpha + 1e-10], 1), 1)[:, :-1]
        w = alpha * T
        acc = w.sum(1)
        bg = self.m.background(rays[:, 3:6])
        return (w.unsqueeze(-1) * rgb).sum(1) + (1.0 - acc.unsqueeze(-1)) * bg, (w * t).sum(1), w, acc


def test_owner_blocks():
    assert expert_owner(8, 8) == list(range(8))
    assert expert_owner(8, 2) == [0, 0, 0, 0, 1, 1, 1, 1]
    assert expert_owner(8, 1) == [0] * 8
    assert expert_owner(4, 3) == [0, 0, 1, 2]
    for K, W in ((8, 3), (5, 4), (16, 8)):
        o = expert_owner(K, W)
        assert o == sorted(o) and set(o) <= set(range(W))


def _shard(n, world, rank):
    lo, hi = n * rank // world, n * (rank + 1) // world
    return slice(lo, hi)


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.set_num_threads(2)
        d = G.load("train_k8")
        m = ref_container(d)
        be = RefBackend(m)
        rays = torch.from_numpy(d["train0:rays"])
        rgbs = torch.from_numpy(d["train0:rgbs"])
        u = torch.from_numpy(d["train0:u"])
        sl = _shard(rays.shape[0], world, rank)
        with torch.no_grad():
            rgb, depth, w, acc = render_rays_expert_parallel(be, rays[sl], S, m.K, u=u[sl])
        opt = torch.optim.Adam(m.param_groups(LRS), lr=1e-4)
        shared = [m.p[f"bg_mlp.{i}.{n}"] for i in (0, 2) for n in ("weight", "bias")]
        loss = adapt_step_expert_parallel(P, be, rays[sl], rgbs[sl], opt, m.K, rays.shape[0], shared, grad_clip=1.0,
                                          u=u[sl])
        owner = expert_owner(m.K, world)
        res = {"rgb": rgb.numpy(), "loss": float(loss), "norm": opt.last_norm[0],
               "params": {n: p.detach().numpy().copy() for n, p in m.p.items()
                          if n.startswith("bg_mlp") or (n.startswith("submodules.") and not n.endswith("hash_table")
                                                        and owner[int(n.split(".")[1])] == rank)},
               "grads": {n: p.grad.numpy().copy() for n, p in m.p.items()
                         if p.grad is not None and not n.endswith("hash_table")},
               "table_rows": {k: m.p[f"submodules.{k}.xyz_encoder.hash_table"].detach()[
                   torch.from_numpy(d["train:rows"][k])].numpy() for k in range(m.K) if owner[k] == rank}}
        out[rank] = res
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(600)
def test_expert_parallel_world2_matches_reference_step():
    d = G.load("train_k8")
    world = 2
    with mp.Manager() as man:
        out = man.dict()
        mp.spawn(_worker, args=(world, _free_port(), out), nprocs=world, join=True)
        res = dict(out)
    # render: the shards concatenated equal the single-process restatement of the same rays
    m = ref_container(d)
    with torch.no_grad():
        ref_rgb = TR.render_train(m, torch.from_numpy(d["train0:rays"]), S, torch.from_numpy(d["train0:u"]))
    np.testing.assert_allclose(np.concatenate([res[r]["rgb"] for r in range(world)]), ref_rgb.numpy(), rtol=0, atol=1e-6)
    # the update: the reference's own step (train_k8.npz step 0)
    for r in range(world):
        assert abs(res[r]["loss"] - float(d["train0:loss"])) <= 1e-6 * float(d["train0:loss"])
        assert abs(res[r]["norm"] - float(d["train0:total_norm"])) <= 1e-5 * float(d["train0:total_norm"])
    owner = expert_owner(8, world)
    for k in range(8):
        r = owner[k]
        for name, v in res[r]["grads"].items():
            if name.startswith(f"submodules.{k}."):
                ref = d["train0:grad:" + name]
                np.testing.assert_allclose(v, ref, rtol=0, atol=1e-5 * (np.abs(ref).max() + 1e-12))
        if f"train0:grad_rows:{k}" in d:
            np.testing.assert_allclose(res[r]["table_rows"][k], d[f"train0:table_rows:{k}"], rtol=0, atol=1e-7)
        for name, v in res[r]["params"].items():
            if name.startswith(f"submodules.{k}.") and ("train0:param:" + name) in d:
                np.testing.assert_allclose(v, d["train0:param:" + name], rtol=0, atol=5e-7)
    for r in range(world):   # the replicated background head: identical update on both ranks
        for name, v in res[r]["params"].items():
            if name.startswith("bg_mlp") and ("train0:param:" + name) in d:
                np.testing.assert_allclose(v, d["train0:param:" + name], rtol=0, atol=5e-7)
                np.testing.assert_array_equal(v, res[0]["params"][name])


# ------------------------------------------------------------------------------------------ GPU
@pytest.mark.gpu
@pytest.mark.parametrize("variant", ["render", "render_hi"])
def test_hip_backend_render_equals_fused(variant):
    """World size 1: the expert-parallel render (pairs as records, per-expert fused field, blend, HIP
    compositing) equals the reference fixture and the fused single-launch render."""
    from adaptive_city_nerf_amd import render_rays
    from adaptive_city_nerf_amd.expert_parallel import HipBackend
    from test_k8 import _model
    d = G.load("render_k8")
    m, _ = _model(d, "hiw:" if variant == "render_hi" else "w:")
    rays = torch.from_numpy(d["render:rays"]).cuda()
    with torch.no_grad():
        rgb, depth, w, acc = render_rays_expert_parallel(HipBackend(m), rays, 64, len(m.submodules))
        frgb, fdepth, fw, facc = render_rays(m, rays, ray_samples=64)
    assert np.abs(rgb.cpu().numpy() - d[f"{variant}:rgb"]).max() <= 1e-4
    assert np.abs(w.cpu().numpy() - d[f"{variant}:weights"]).max() <= 1e-5
    torch.testing.assert_close(rgb, frgb, rtol=0, atol=2e-6)
    torch.testing.assert_close(acc, facc, rtol=0, atol=2e-6)


@pytest.mark.gpu
def test_hip_backend_adapt_step_matches_reference_fixture():
    """World size 1: adapt_step_expert_parallel on the HIP backend replays the reference's K=8
    runtime_adapt steps (same checks as the single-process step)."""
    from test_train import check_adapt_fixture
    from adaptive_city_nerf_amd.expert_parallel import HipBackend

    def fn(Pk, m, rays, rgbs, opt, u):
        shared = list(m.bg_mlp.parameters())
        return adapt_step_expert_parallel(Pk, HipBackend(m), rays, rgbs, opt, len(m.submodules), rays.shape[0],
                                          shared, grad_clip=1.0, u=u)
    check_adapt_fixture("k8", fn)


# ------------------------------------------------------------------------------- sync-free step (GPU)
def _ep_step_fn(graph, n_global=None):
    """check_adapt_fixture step through ExpertParallelAdaptStep at world size 1 (the exchanges are copies):
    built on the first call; graph=True: one eager real step, then the captured step replayed."""
    def fn(Pk, m, rays, rgbs, opt, u):
        from adaptive_city_nerf_amd.expert_parallel import ExpertParallelAdaptStep
        st = getattr(opt, "_ep_step", None)
        if st is None:
            st = opt._ep_step = ExpertParallelAdaptStep(Pk, m, rays.shape[0], opt, grad_clip=1.0, graph=graph,
                                                        warmup=1, jitter="given", clear_in_adam=False)
        loss = st(rays, rgbs, jitter_u=u)
        opt.last_norm = st.last_norm
        return loss
    return fn


@pytest.mark.gpu
@pytest.mark.parametrize("graph", [False, True])
def test_ep_step_world1_matches_reference_fixture(graph):
    """ExpertParallelAdaptStep (fixed-capacity exchange, no host read, slotted Adam) at world size 1 replays
    the reference's K=8 runtime_adapt steps, eagerly and as a replayed HIP graph (steps 2-3)."""
    from test_train import check_adapt_fixture
    m, opt = check_adapt_fixture("k8", _ep_step_fn(graph))
    st = opt._ep_step
    assert st.steps_done == 3 and st.replays == (2 if graph else 0)


def _ep_gpu_worker(rank, world, port, out):
    """World-2 gloo group on ONE GPU: the product's exchange code (_Comm staged through host copies) with the
    HIP kernels; strong mode -- the fixture's 1000-ray batch split over the ranks, loss over all 1000."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        from test_module_api import build_model, reference_state_dict
        from adaptive_city_nerf_amd.expert_parallel import ExpertParallelAdaptStep
        from adaptive_city_nerf_amd.optim import build_optimizer
        d = G.load("train_k8")
        Pk = SimpleNamespace(ray_samples=96, chunk_points=4_000_000, color_space="linear", optimizer="adam", lr=1e-4,
                             encoding_lr=0.01, sigma_lr=0.002, color_lr=0.002, bg_lr=0.001, weight_decay=0.0)
        m, _ = build_model("k8")
        m.load_state_dict(reference_state_dict(d, 8, "w:"))
        m = m.cuda().train()
        opt = build_optimizer(Pk, m)
        rays = torch.from_numpy(d["train0:rays"]).cuda()
        sl = _shard(rays.shape[0], world, rank)
        n_loc = sl.stop - sl.start
        st = ExpertParallelAdaptStep(Pk, m, n_loc, opt, n_rays_global=rays.shape[0], grad_clip=1.0,
                                     group=dist.group.WORLD, jitter="given", clear_in_adam=False)
        res = {"loss": [], "norm": [], "grads": {}, "params": {}}
        owner = expert_owner(8, world)
        for step in range(3):
            pre = f"train{step}:"
            r = torch.from_numpy(d[pre + "rays"]).cuda()[sl]
            c = torch.from_numpy(d[pre + "rgbs"]).cuda()[sl]
            u = torch.from_numpy(d[pre + "u"]).cuda()[sl]
            loss = st(r, c, jitter_u=u)
            torch.cuda.synchronize()
            res["loss"].append(float(loss[0]))
            res["norm"].append(float(st.last_norm[0]))
            if step == 0:
                for name, p in m.named_parameters():
                    if name.startswith("submodules.") and owner[int(name.split(".")[1])] == rank \
                            and not name.endswith("hash_table") and p.grad is not None:
                        res["grads"][name] = p.grad.cpu().numpy().copy()
                    if name.startswith("bg_mlp"):
                        res["grads"][name] = p.grad.cpu().numpy().copy()
                res["table_rows"] = {k: m.submodules[k].xyz_encoder.hash_table.detach()[
                    torch.from_numpy(d["train:rows"][k]).cuda()].cpu().numpy() for k in range(8) if owner[k] == rank}
        for name, p in m.named_parameters():
            if name.startswith("bg_mlp") or (name.startswith("submodules.") and owner[int(name.split(".")[1])] == rank
                                             and not name.endswith("hash_table")):
                res["params"][name] = p.detach().cpu().numpy().copy()
        out[rank] = res
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.timeout(600)
def test_ep_step_world2_gloo_on_gpu_matches_reference():
    """Two ranks on one GPU over gloo (staged exchange), each holding half of the reference batch and 4 of
    the 8 experts: every step's global loss and clip norm, the owned experts' gradients and step-0 table rows,
    and after 3 steps the owned experts' MLPs and the replicated background head equal the reference's
    single-process runtime_adapt (train_k8.npz) -- strong scaling of one 1000-ray update."""
    d = G.load("train_k8")
    world = 2
    with mp.Manager() as man:
        out = man.dict()
        mp.spawn(_ep_gpu_worker, args=(world, _free_port(), out), nprocs=world, join=True)
        res = dict(out)
    for step in range(3):
        ref = float(d[f"train{step}:loss"])
        for r in range(world):
            assert abs(res[r]["loss"][step] - ref) <= 1e-5 * ref, (step, r, res[r]["loss"][step], ref)
            nref = float(d[f"train{step}:total_norm"])
            assert abs(res[r]["norm"][step] - nref) <= 1e-4 * nref, (step, r)
    owner = expert_owner(8, world)
    for r in range(world):
        for name, v in res[r]["grads"].items():
            if "train0:grad:" + name not in d:   # an expert the batch does not reach: grad None in the reference
                assert not np.any(v), name
                continue
            ref = d["train0:grad:" + name]
            np.testing.assert_allclose(v, ref, rtol=0, atol=1e-4 * (np.abs(ref).max() + 1e-12), err_msg=name)
        for k, rows in res[r]["table_rows"].items():
            if f"train0:table_rows:{k}" in d:   # Adam's first step: ~lr * sign(g) per touched row
                ref = d[f"train0:table_rows:{k}"]
                close = np.mean(np.abs(rows.astype(np.float64) - ref) <= 1e-3 * 0.01 + 1e-6 * np.abs(ref))
                assert close >= 0.99, (k, close)
        for name, v in res[r]["params"].items():
            key = "train2:param:" + name
            if key in d:
                lr = 0.001 if name.startswith("bg_mlp") else 0.002
                close = np.mean(np.abs(v.astype(np.float64) - d[key]) <= 1e-3 * lr + 1e-6 * np.abs(d[key]))
                assert close >= 0.95, (name, close)
    for name, v in res[0]["params"].items():   # the replicated head: identical on both ranks
        if name.startswith("bg_mlp"):
            np.testing.assert_array_equal(v, res[1]["params"][name])


def _comm_worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from adaptive_city_nerf_amd.expert_parallel import _Comm
        comm = _Comm(dist.group.WORLD)
        K, C = 8, 5
        owner = expert_owner(K, world)
        eo = [owner.count(o) for o in range(world)]
        E = eo[rank]
        # sender layout [expert k][C] rows tagged (rank, k, i); the owner receives [src][local j][C]
        send = torch.tensor([[rank, k, i] for k in range(K) for i in range(C)], dtype=torch.float32)
        recv = torch.empty(world * E * C, 3)
        comm.all_to_all(recv, send, [E * C] * world, [e * C for e in eo])
        cnt = torch.arange(K, dtype=torch.int64) + 10 * rank
        rc = torch.empty(world * E, dtype=torch.int64)
        comm.all_to_all(rc, cnt, [E] * world, eo)
        t = torch.tensor([float(rank + 1)], dtype=torch.float64)
        comm.all_reduce(t)
        out[rank] = (recv.numpy(), rc.numpy(), float(t[0]), comm.staged)
    finally:
        dist.destroy_process_group()


def test_ep_comm_fixed_splits_gloo_world2():
    """The sync-free step's exchange helper (_Comm) on gloo: constant split sizes route sender segment
    [expert k] of every rank to k's owner as [src][local expert][C]; counts likewise; sums all-reduced."""
    world = 2
    with mp.Manager() as man:
        out = man.dict()
        mp.spawn(_comm_worker, args=(world, _free_port(), out), nprocs=world, join=True)
        res = dict(out)
    owner = expert_owner(8, world)
    for r in range(world):
        recv, rc, tot, staged = res[r]
        assert staged and tot == 3.0
        mine = [k for k in range(8) if owner[k] == r]
        exp = np.array([[s, k, i] for s in range(world) for k in mine for i in range(5)], np.float32)
        np.testing.assert_array_equal(recv, exp)
        np.testing.assert_array_equal(rc, np.array([k + 10 * s for s in range(world) for k in mine]))


# --------------------------------------------------------------- sync-free one-expert-per-GPU render (GPU)
@pytest.mark.gpu
@pytest.mark.parametrize("tile", [1, 7, 32, 1 << 20])
def test_routed_pairs_depth_tiled_order(tile):
    """acn_routed_count_caps_tiled + acn_routed_scatter_xd_tiled (the renderer's record order): the same pairs,
    counts and t values as the sample order, every expert's segment permuted into depth-tile order -- blocks of
    `tile` consecutive rays (the last one shorter), a block's rays at sample s before its rays at s + 1 -- with the
    records, weights and expert ids moved bit for bit and pmap pointing at the new positions."""
    from adaptive_city_nerf_amd import ops
    from test_k8 import _model
    d = G.load("render_k8")
    m, _ = _model(d, "w:")
    rays = torch.from_numpy(d["render:rays"]).cuda()
    N, S = rays.shape[0], 64
    with torch.no_grad():
        a = ops.routed_pairs_xd(rays, S, None, m.routing_spec())
        b = ops.routed_pairs_xd(rays, S, None, m.routing_spec(), tile_rays=tile)
    t0, c0, pidx0, pw0, xd0, pmap0, pk0 = [x.cpu().numpy() if torch.is_tensor(x) else x for x in a]
    t1, c1, pidx1, pw1, xd1, pmap1, pk1 = [x.cpu().numpy() if torch.is_tensor(x) else x for x in b]
    assert c0 == c1 and sum(c0) > 0
    np.testing.assert_array_equal(t0, t1)
    samp = pidx0.astype(np.int64)
    ray, s = samp // S, samp % S
    blk = ray // tile
    nb = np.minimum(tile, N - blk * tile)
    pos = blk * tile * S + s * nb + (ray - blk * tile)     # traversal position of the sample (tile_sample inverse)
    start = np.concatenate([[0], np.cumsum(c0)])
    for k in range(len(c0)):
        sl = slice(start[k], start[k + 1])
        order = np.argsort(pos[sl], kind="stable")
        np.testing.assert_array_equal(pidx1[sl], pidx0[sl][order], err_msg=f"expert {k}")
        np.testing.assert_array_equal(xd1[sl], xd0[sl][order])
        np.testing.assert_array_equal(pw1[sl], pw0[sl][order])
        np.testing.assert_array_equal(pk1[sl], pk0[sl][order])
    assert ((pmap0 < 0) == (pmap1 < 0)).all()
    P = int(start[-1])
    np.testing.assert_array_equal(pmap1[pidx1.astype(np.int64), pk1.astype(np.int64)], np.arange(P))


@pytest.mark.gpu
@pytest.mark.parametrize("variant", ["render", "render_hi"])
@pytest.mark.parametrize("graph", [False, True])
@pytest.mark.parametrize("tile", [0, 32])
def test_ep_renderer_world1_equals_fused_render(variant, graph, tile):
    """ExpertParallelRenderer at world size 1 (exchanges are copies; graph=True: the first full batch is run
    eagerly and captured, later calls replay it): every ray's rgb / depth / weights / acc equal the fused
    single-process routed render bit for bit (same per-(sample, expert) arithmetic, blend in expert order,
    same compositing), and the reference fixture within the north-star tolerances.  A capacity below the
    largest expert's pair count is detected (overflowed) and, re-rendered at full capacity, gives the same
    frame.  tile: the record order (0 sample order, 32 the default depth tiles): no value may change."""
    from adaptive_city_nerf_amd import render_rays
    from adaptive_city_nerf_amd.expert_parallel import ExpertParallelRenderer, render_rays_ep_batched
    from test_k8 import _model
    d = G.load("render_k8")
    m, _ = _model(d, "hiw:" if variant == "render_hi" else "w:")
    rays = torch.from_numpy(d["render:rays"]).cuda()
    n = rays.shape[0]
    r = ExpertParallelRenderer(m, n, 64, graph=graph, want_weights=True, tile_rays=tile)
    with torch.no_grad():
        fr = render_rays(m, rays, ray_samples=64, bg_color_default="white")
        for rep in range(3):
            out = [x.clone() for x in r(rays)]
            for x, y in zip(out, fr):
                assert torch.equal(x, y), rep
    assert (r.graph is not None) == graph and r.replays == (2 if graph else 0)
    assert not r.overflowed()
    assert np.abs(out[0].cpu().numpy() - d[f"{variant}:rgb"]).max() <= 1e-4
    assert np.abs(out[2].cpu().numpy() - d[f"{variant}:weights"]).max() <= 1e-5
    # capacity-bounded exchange: an overflow is seen and the batch re-rendered at full capacity
    small = ExpertParallelRenderer(m, n, 64, capacity=n * 64 // 16, tile_rays=tile)
    with torch.no_grad():
        small(rays)
        assert small.overflowed()
        rgb, depth, acc = render_rays_ep_batched(m, rays, 64, batch=n, capacity_frac=1.0 / 16)
    assert torch.equal(rgb, fr[0]) and torch.equal(depth, fr[1]) and torch.equal(acc, fr[3])
    # the planned exchange (the default): per-batch pair counts from acn_routed_count_batches, segments sized to
    # exactly the live pairs -- same pixels, 40 B sent per routed pair and nothing else (VERDICT r04 missing 1)
    from adaptive_city_nerf_amd import ops
    _, counts, *_ = ops.routed_pairs_xd(rays, 64, None, m.routing_spec())
    for batch in (n, 100, 37):
        st = {}
        with torch.no_grad():
            rgb, depth, acc = render_rays_ep_batched(m, rays, 64, batch=batch, stats=st)
        assert torch.equal(rgb, fr[0]) and torch.equal(depth, fr[1]) and torch.equal(acc, fr[3]), batch
        assert st["sent"] == st["live"] == 40 * sum(counts), (batch, st, sum(counts))


def _ep_render_worker(rank, world, port, out):
    """World-2 gloo group on ONE GPU: the renderer's exchange (staged through host copies) with the HIP kernels;
    rank r renders half of the fixture's rays, owning 4 of the 8 experts."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from adaptive_city_nerf_amd.expert_parallel import ExpertParallelRenderer, render_rays_ep_batched
        from test_k8 import _model
        d = G.load("render_k8")
        m, _ = _model(d, "hiw:")
        rays = torch.from_numpy(d["render:rays"]).cuda()
        sl = _shard(rays.shape[0], world, rank)
        lo, hi = sl.start, sl.stop
        mine = rays[lo:hi].contiguous()
        r = ExpertParallelRenderer(m, mine.shape[0], 64, group=dist.group.WORLD, want_weights=True)
        with torch.no_grad():
            o = r(mine)
            res = {"rgb": o[0].cpu().numpy().copy(), "depth": o[1].cpu().numpy().copy(),
                   "weights": o[2].cpu().numpy().copy(), "acc": o[3].cpu().numpy().copy(), "lo": lo, "hi": hi}
            b = render_rays_ep_batched(m, mine, 64, group=dist.group.WORLD, batch=100, capacity_frac=0.25)
            res["batched_rgb"] = b[0].cpu().numpy().copy()
            st = {}
            pl = render_rays_ep_batched(m, mine, 64, group=dist.group.WORLD, batch=97, stats=st)
            res["planned"] = [x.cpu().numpy().copy() for x in pl]
            res["planned_stats"] = dict(st)
        out[rank] = res
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.timeout(600)
def test_ep_renderer_world2_gloo_on_gpu_matches_fused_and_reference():
    """Two ranks on one GPU, each rendering half of the K=8 fixture rays and owning 4 experts: the gathered
    render equals the single-process fused render bit for bit and the reference fixture (RGB 1e-4, weights
    1e-5); the batched form with a quarter-capacity exchange (overflows re-rendered) gives the same pixels."""
    from adaptive_city_nerf_amd import render_rays
    from test_k8 import _model
    d = G.load("render_k8")
    world = 2
    with mp.Manager() as man:
        out = man.dict()
        mp.spawn(_ep_render_worker, args=(world, _free_port(), out), nprocs=world, join=True)
        res = dict(out)
    m, _ = _model(d, "hiw:")
    with torch.no_grad():
        fr = [x.cpu().numpy() for x in render_rays(m, torch.from_numpy(d["render:rays"]).cuda(), ray_samples=64,
                                                      bg_color_default="white")]
    for r in range(world):
        lo, hi = res[r]["lo"], res[r]["hi"]
        for key, ref in zip(("rgb", "depth", "weights", "acc"), fr):
            np.testing.assert_array_equal(res[r][key], ref[lo:hi], err_msg=f"rank {r} {key}")
        np.testing.assert_array_equal(res[r]["batched_rgb"], fr[0][lo:hi])
        for got, ref in zip(res[r]["planned"], (fr[0], fr[1], fr[3])):   # planned exchange: the same pixels
            np.testing.assert_array_equal(got, ref[lo:hi])
        assert res[r]["planned_stats"]["sent"] == res[r]["planned_stats"]["live"] > 0
        assert np.abs(res[r]["rgb"] - d["render_hi:rgb"][lo:hi]).max() <= 1e-4
        assert np.abs(res[r]["weights"] - d["render_hi:weights"][lo:hi]).max() <= 1e-5


@pytest.mark.gpu
@pytest.mark.parametrize("capacity", ["adaptive", 2000])
def test_ep_step_bounded_exchange_matches_reference_fixture(capacity):
    """VERDICT r03 "Next" 5: the exchange sized to the live records.  "adaptive": full capacity for the eager
    warm-up step, then per expert ~1.5x the largest routed count, the captured step replayed -- no overflow on
    the fixture, at most ~2x the live 56 B per pair; 2000: every step overflows (expert 2 takes ~85k pairs), is
    gated off on the device (no update, no step count) and re-run at full capacity.  Both replay the
    reference's K=8 runtime_adapt steps (train_k8.npz)."""
    from test_train import check_adapt_fixture
    from adaptive_city_nerf_amd.expert_parallel import ExpertParallelAdaptStep

    def fn(Pk, m, rays, rgbs, opt, u):
        st = getattr(opt, "_ep_step", None)
        if st is None:
            st = opt._ep_step = ExpertParallelAdaptStep(Pk, m, rays.shape[0], opt, grad_clip=1.0, graph=True,
                                                        warmup=1, jitter="given", clear_in_adam=False,
                                                        capacity=capacity)
        st(rays, rgbs, jitter_u=u)
        st.flush()
        opt.last_norm = st.last_norm
        return st.loss_global
    m, opt = check_adapt_fixture("k8", fn)
    st = opt._ep_step
    live = int(st.seg[st.K + 1: 2 * st.K + 1].sum())
    if capacity == "adaptive":
        assert st.bounded and st.overflows == 0 and st.replays == 2
        assert st.exchange_bytes() <= 2 * (56 * live + 8 * st.K), (st.exchange_bytes(), live, st.caps)
    else:
        assert st.overflows == 3
