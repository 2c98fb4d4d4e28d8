"""Expert-parallel offline meta-training (meta_train.train_step(group=)): world size 2
over gloo on the CPU.  Rank r takes the regions whose experts it owns (expert_parallel.expert_owner:
regions 0 and 2 of the fixture land on ranks 0 and 1), consumes the training jitter the single
process would have used for those renders, and after the outer update every owned expert and the
all-reduced background head must equal the reference's own single-process step
(tests/golden/meta_{fomaml,maml}.npz).  The product's train_step / task_adapt / meta_update run
unchanged; only the expert render (the HIP kernels) is replaced by the CPU restatement
(oracle/meta_ref.render_fast) evaluated on the product model's own parameters."""
import os
import socket
from types import SimpleNamespace

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import goldens as G
from oracle import meta_ref as MR
from oracle import oracle as O
from oracle import train_ref as TR

S = 16


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


class ModelView:
    """train_ref.RefContainer's surface over a MetaContainer's own (shared, not copied) parameters."""

    def __init__(self, model):
        sc = G.scene()["masks"][G.MASK["k4"]]
        self.p = dict(model.named_parameters())
        self.res = torch.as_tensor(O.level_resolutions(16, 16, 4096), dtype=torch.int64)
        self.log2T = 20
        self.mins = torch.tensor(sc["mins"], dtype=torch.float32)
        self.ext = torch.stack([s.aabb_extent for s in model.submodules])

    background = TR.RefContainer.background


def _u_for_rank(d, algo, owner, rank):
    """The jitter the single process drew for this rank's renders, in this rank's call order."""
    u = list(torch.from_numpy(d["u"]))
    if algo == "maml":
        u = u[int(d["adapt_n_u"]):]   # the fixture's standalone task_adapt came first
    per_region = 2 + 1                  # inner_iter renders + the query render
    mine = []
    for i, cid in enumerate(d["region_order"].tolist()):
        if owner[cid] == rank:
            mine += u[i * per_region:(i + 1) * per_region]
    return iter(mine)


def _worker(rank, world, port, algo, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.set_num_threads(2)
        from test_module_api import build_model, reference_state_dict
        from adaptive_city_nerf_amd import meta_train as MT
        from adaptive_city_nerf_amd.expert_parallel import expert_owner
        from adaptive_city_nerf_amd.optim import build_optimizer
        d = G.load(f"meta_{algo}")
        m, _ = build_model("k4")
        m.load_state_dict(reference_state_dict(d, 4, "w:"))
        owner = expert_owner(4, world)
        us = _u_for_rank(d, algo, owner, rank)
        view = ModelView(m)

        def cpu_compute_loss(P, model, data, params=None, active_module=None, **kw):
            pred = MR.render_fast(view, data["rays"], S, next(us), active_module, params or {})
            return MR.mse_linear(pred, data["rgbs"])
        MT.compute_loss = cpu_compute_loss
        P = SimpleNamespace(algo=algo, ray_samples=S, color_space="linear", optimizer="adam", lr=1e-4, encoding_lr=0.01,
                            sigma_lr=0.002, color_lr=0.002, bg_lr=0.001, weight_decay=0.0, inner_lr=0.05, inner_iter=2,
                            grad_clip=1.0, seed=0, print_step=10 ** 9)
        opt = build_optimizer(P, m, fused=False)
        task_data = {cid: [{part: {"rays": torch.from_numpy(d[f"task{cid}:{part}:rays"]),
                                   "rgbs": torch.from_numpy(d[f"task{cid}:{part}:rgbs"])}
                            for part in ("support", "query")}] for cid in (0, 2)}
        import contextlib
        import io
        with contextlib.redirect_stdout(io.StringIO()):
            res = MT.train_step(P, 1, m, opt, task_data, group=dist.group.WORLD)
        sd = {n: p.detach().numpy().copy() for n, p in m.named_parameters() if not n.endswith("hash_table")}
        rows = torch.from_numpy(d["rows"])
        tabs = {k: m.submodules[k].xyz_encoder.hash_table.detach()[rows[k]].numpy().copy() for k in range(4)}
        out[rank] = {"params": sd, "tables": tabs, "loss_out": res["loss_out"]}
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(600)
@pytest.mark.parametrize("algo", ["fomaml", "maml"])
def test_meta_train_step_world2_matches_reference(algo):
    from adaptive_city_nerf_amd.expert_parallel import expert_owner
    d = G.load(f"meta_{algo}")
    world = 2
    with mp.Manager() as man:
        out = man.dict()
        mp.spawn(_worker, args=(world, _free_port(), algo, out), nprocs=world, join=True)
        res = dict(out)
    owner = expert_owner(4, world)
    assert sorted({owner[c] for c in (0, 2)}) == [0, 1]          # both ranks hold a region
    assert res[0]["loss_out"] == pytest.approx(res[1]["loss_out"], rel=1e-6)
    for cid in (0, 2):
        r = owner[cid]
        for name, v in res[r]["params"].items():
            if name.startswith(f"submodules.{cid}.") and "after:" + name in d:
                np.testing.assert_allclose(v, d["after:" + name], rtol=1e-4, atol=1e-6, err_msg=name)
        np.testing.assert_allclose(res[r]["tables"][cid], d[f"after_table_rows:{cid}"], rtol=1e-4, atol=1e-6)
    for r in range(world):
        for name, v in res[r]["params"].items():
            if name.startswith("bg_mlp"):
                np.testing.assert_allclose(v, d["after:" + name], rtol=1e-4, atol=1e-6, err_msg=name)
                np.testing.assert_array_equal(v, res[0]["params"][name])
