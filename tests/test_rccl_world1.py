"""The RCCL branch of the expert-parallel layouts, run once on one GPU (VERDICT r04 missing 3).

A world-size-1 ``nccl`` process group (RCCL) with ``expert_parallel.FORCE_COLLECTIVES`` (and, for the replicated
layout, ``parallel.FORCE_COLLECTIVES``): every exchange of
ExpertParallelRenderer and ExpertParallelAdaptStep goes through ``dist.all_to_all_single`` / ``all_reduce`` /
``all_gather_into_tensor`` on RCCL instead of the world-1 plain copies -- eager, and captured in a HIP graph
(the ``--ep-graph`` path: RCCL collectives inside a graph).  Every result must be bitwise the plain-copy one
and match the reference's K = 8 fixtures (render_k8.npz: RGB 1e-4, weights 1e-5; train_k8.npz: the
runtime_adapt steps).  The training step's first loss and MLP weight gradients are bitwise the plain-copy
step's; its later steps agree within the fixture tolerance (the table gradients are float-atomic sums).  Reference: pipelines/online_stage/runtime_adapt.py:286-309,
models/inr/meta_container.py:300-337."""
import os

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import goldens as G
from test_expert_parallel import _free_port

pytestmark = pytest.mark.gpu


def _render_all(m, rays, EP):
    out = {}
    with torch.no_grad():
        for graph in (False, True):
            r = EP.ExpertParallelRenderer(m, rays.shape[0], 64, group=dist.group.WORLD if EP.FORCE_COLLECTIVES
                                          else None, graph=graph, want_weights=True)
            for rep in range(3):   # graph: the eager call, the capture, then replays
                o = [x.clone() for x in r(rays)]
            out[f"graph{int(graph)}"] = [x.cpu().numpy() for x in o]
            out[f"replays{int(graph)}"] = r.replays
            out[f"closed{int(graph)}"] = r.close()   # the captured graph (and its RCCL resources) released
        st = {}
        p = EP.render_rays_ep_batched(m, rays, 64, group=dist.group.WORLD if EP.FORCE_COLLECTIVES else None,
                                      batch=200, stats=st)
        out["planned"] = [x.cpu().numpy() for x in p]
    return out


def _train_all(EP, graph):
    """The reference's K = 8 runtime_adapt steps (check_adapt_fixture asserts loss, clip norm, gradients and
    parameters against train_k8.npz); returns the first step's loss and MLP weight gradients (exact: the
    forward and the per-expert [dW | db] partial sums have a fixed order) and the per-step losses.  Later steps
    are compared within the fixture's tolerance only: the table gradients are float-atomic scatter-adds."""
    import hashlib
    from test_train import check_adapt_fixture
    rec = {"loss": []}

    def fn(Pk, m, rays, rgbs, opt, u):
        st = getattr(opt, "_ep_step", None)
        if st is None:
            st = opt._ep_step = EP.ExpertParallelAdaptStep(
                Pk, m, rays.shape[0], opt, grad_clip=1.0, graph=graph, warmup=1, jitter="given",
                clear_in_adam=False, group=dist.group.WORLD if EP.FORCE_COLLECTIVES else None)
        st(rays, rgbs, jitter_u=u)
        st.flush()
        opt.last_norm = st.last_norm
        rec["loss"].append(float(st.loss_global))
        if "dw0" not in rec:
            rec["dw0"] = hashlib.sha1(st.dw.detach().cpu().numpy().tobytes()).hexdigest()
        return st.loss_global
    m, opt = check_adapt_fixture("k8", fn)
    st = opt._ep_step
    res = rec, st.replays, st.comm.direct
    rec["closed"] = st.close()
    return res


def _replicated_image():
    """parallel.render_image_sharded (the C3/C4 replicated layout) with its collectives forced through the
    world-size-1 nccl group: the all_gather_into_tensor of the rendered rows and the fp64 PSNR all_reduce
    (runtime_adapt.py:152-157) on RCCL, against render_image and the whole frame's PSNR in one process."""
    from adaptive_city_nerf_amd import parallel as P
    from adaptive_city_nerf_amd import render_image
    from test_module_api import build_model, reference_state_dict
    m, gbox = build_model("k4")
    d = G.load("render_k4")
    m.load_state_dict(reference_state_dict(d, len(m.submodules), "hiw:"))
    m = m.cuda().eval()
    cam = G.scene()["val_cam0"]
    H, W = [int(v) for v in d["image:hw"]]
    intr = (torch.tensor(cam["intrinsics"], dtype=torch.float32) / 32).tolist()
    kw = dict(H=H, W=W, fx=intr[0], fy=intr[1], cx=intr[2], cy=intr[3], c2w=torch.tensor(cam["c2w"]), scene_box=gbox,
              ray_samples=32)
    with torch.no_grad():
        img0, _, acc0 = render_image(m, **kw)
    gt = torch.rand(H, W, 3, device="cuda", generator=torch.Generator(device="cuda").manual_seed(5))
    sse, cnt = P.local_sse(img0.view(-1, 3), gt.view(-1, 3), "linear")
    P.FORCE_COLLECTIVES = True
    try:
        img1, _, acc1, psnr = P.render_image_sharded(m, gt_srgb=gt, group=dist.group.WORLD, **kw)
    finally:
        P.FORCE_COLLECTIVES = False
    return {"img_equal": bool(torch.equal(img0, img1)), "acc_equal": bool(torch.equal(acc0, acc1)),
            "img_vs_fixture": float(np.abs(img1.cpu().numpy() - d["image:rgb"]).max()),
            "psnr": psnr, "psnr_one": P.psnr_reduce(sse, cnt, "cuda")}


def _say(msg):
    print(f"[rccl-world1] {msg}", flush=True)


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    _say("init_process_group(nccl)")
    dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", 0))
    try:
        from adaptive_city_nerf_amd import expert_parallel as EP
        from adaptive_city_nerf_amd import render_rays
        from test_k8 import _model
        assert dist.get_backend() == "nccl"
        d = G.load("render_k8")
        m, _ = _model(d, "hiw:")
        rays = torch.from_numpy(d["render:rays"]).cuda()
        with torch.no_grad():
            fused = [x.cpu().numpy() for x in render_rays(m, rays, ray_samples=64, bg_color_default="white")]
        res = {"fused": fused}
        EP.FORCE_COLLECTIVES = False
        _say("plain-copy render")
        res["plain_render"] = _render_all(m, rays, EP)
        _say("plain-copy step")
        res["plain_train"] = _train_all(EP, graph=True)
        EP.FORCE_COLLECTIVES = True
        _say("RCCL render (eager, graph, planned)")
        res["rccl_render"] = _render_all(m, rays, EP)
        _say("RCCL step, eager")
        res["rccl_train_eager"] = _train_all(EP, graph=False)
        _say("RCCL step, graph-captured")
        res["rccl_train_graph"] = _train_all(EP, graph=True)
        _say("replicated layout: all-gather of the rendered rows + fp64 PSNR all-reduce over RCCL")
        res["replicated"] = _replicated_image()
        _say("done")
        out[rank] = res
    finally:
        from adaptive_city_nerf_amd import expert_parallel as EP
        EP.FORCE_COLLECTIVES = False
        torch.cuda.synchronize()
    # RCCL keeps a communicator's resources until every graph that captured one of its collectives is destroyed,
    # and ncclCommDestroy waits for them: the objects above released their graphs (close()), and EP.shutdown
    # releases any still alive, then destroys the group -- bounded, so a teardown that does not return fails the
    # test instead of hanging it (round 5 left with os._exit(0) here: DESIGN.md §4l)
    _say("destroy_process_group")
    ok = EP.shutdown(timeout=120.0)
    out["teardown"] = ok
    _say(f"teardown returned: {ok}")
    if not ok:
        os._exit(3)


@pytest.mark.timeout(900)
def test_rccl_world1_ep_render_and_step_equal_plain_copies_and_fixtures():
    d = G.load("render_k8")
    ctx = mp.get_context("spawn")
    with ctx.Manager() as man:
        out = man.dict()
        p = ctx.Process(target=_worker, args=(0, 1, _free_port(), out))
        p.start()
        p.join(800)
        if p.is_alive():   # the worker's exit (interpreter teardown) did not return
            p.kill()
            p.join()
            pytest.fail("the RCCL worker did not exit after destroy_process_group")
        res = dict(out)
    assert res.get("teardown") is True, "destroy_process_group did not return within 120 s"
    assert p.exitcode == 0, p.exitcode
    res = res[0]
    fused = res["fused"]
    for tag in ("plain_render", "rccl_render"):
        r = res[tag]
        for g in ("graph0", "graph1"):
            for name, a, b in zip(("rgb", "depth", "weights", "acc"), r[g], fused):
                np.testing.assert_array_equal(a, b, err_msg=f"{tag} {g} {name}")
            assert np.abs(r[g][0] - d["render_hi:rgb"]).max() <= 1e-4
            assert np.abs(r[g][2] - d["render_hi:weights"]).max() <= 1e-5
        assert r["replays1"] == 2 and r["replays0"] == 0
        assert r["closed1"] == 1 and r["closed0"] == 0
        for a, b in zip(r["planned"], (fused[0], fused[1], fused[3])):
            np.testing.assert_array_equal(a, b, err_msg=f"{tag} planned")
    rep = res["replicated"]
    assert rep["img_equal"] and rep["acc_equal"], rep
    assert rep["img_vs_fixture"] <= 1e-4, rep
    assert rep["psnr"] == rep["psnr_one"] and np.isfinite(rep["psnr"]), rep
    plain, _, direct0 = res["plain_train"]
    assert not direct0
    for tag in ("rccl_train_eager", "rccl_train_graph"):
        rec, replays, direct = res[tag]
        assert direct, tag                                  # the exchanges went through RCCL
        assert replays == (2 if tag.endswith("graph") else 0), (tag, replays)
        assert rec["closed"] == (1 if tag.endswith("graph") else 0), tag
        assert rec["loss"][0] == plain["loss"][0], (tag, rec["loss"], plain["loss"])    # bitwise: step 0
        assert rec["dw0"] == plain["dw0"], tag                                          # bitwise: step-0 MLP dW
        np.testing.assert_allclose(rec["loss"], plain["loss"], rtol=1e-5)
