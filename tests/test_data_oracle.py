"""Data layer on the CPU: pin oracle/data_ref.py against the reference's own
RamRaysDataset / TaskDataset outputs (tests/golden/data_tasks.npz, make_golden.py gen_data), and check
the host half of adaptive_city_nerf_amd.data (metadata layout, episode sampling) without a GPU.

Everything here is index / byte work: bit-exact (ray tables are compared by SHA-256 of their bytes).
"""
import hashlib

import numpy as np
import pytest
import torch

import goldens as G
from oracle import data_ref as D


def _tables():
    d = G.load("data_tasks")
    return d, {r: D.ray_table(d["images"], G.data_masks(d, r), d["c2w"], d["intrinsics"], d["image_index"],
                              d["box_aabbs"][r], tuple(d[f"r{r}_override"])) for r in (0, 2)}


@pytest.mark.parametrize("region", [0, 2])
def test_oracle_ray_table_is_the_reference_bytes(region):
    d, tabs = _tables()
    for key, arr in zip(("rays", "rgbs", "img"), tabs[region]):
        assert hashlib.sha256(np.ascontiguousarray(arr).tobytes()).hexdigest() == str(d[f"r{region}_{key}_sha"]), key
    np.testing.assert_array_equal(tabs[region][0][::61], d[f"r{region}_rays_sample"])


@pytest.mark.parametrize("name", list(G.TASK_CASES))
def test_oracle_routing_reproduces_reference_pools(name):
    d, tabs = _tables()
    region, kw = G.task_kwargs(d, name)
    rays = tabs[region][0]
    cid, flags = D.route(rays, d[f"t_{name}_aabb"], kw["cells"], kw.get("assignment_checkpoint", 0.7),
                         kw["routing_policy"])
    assert int((flags & 1).sum()) == int(d[f"t_{name}_n_valid"])
    pools = D.replay_pools(D.bins(cid, flags, int(np.prod(kw["cells"]))), kw["seed"])
    for got, want in zip(pools, G.split_pools(d, name)):
        np.testing.assert_array_equal(got, want)


def _fake_table(d, region):
    class T:
        pass
    t = T()
    img = torch.from_numpy(d[f"r{region}_img"].astype(np.int32))
    t._img_indices = img
    t._rays = torch.zeros(img.numel(), 8)
    t._rgbs = torch.zeros(img.numel(), 3)
    return t


@pytest.mark.parametrize("name", list(G.TASK_CASES))
def test_task_sampling_host_logic_matches_reference(name):
    """TaskDataset given the reference's bins (recovered from its pools by inverting the seeded
    permutations): same pools, eligible cells and episodes (cell pick, image choice, per-image cap,
    image-disjoint fallback) draw for draw."""
    from adaptive_city_nerf_amd.data import TaskDataset
    d = G.load("data_tasks")
    region, kw = G.task_kwargs(d, name)
    kw.setdefault("region_bounds", tuple(map(tuple, d[f"t_{name}_aabb"].tolist())))
    bins = [torch.from_numpy(b) for b in D.unreplay_pools(G.split_pools(d, name), kw["seed"])]
    td = TaskDataset(_fake_table(d, region), cell_id=region, bins=bins, **kw)
    for got, want in zip(td._cell_flat_idx, G.split_pools(d, name)):
        np.testing.assert_array_equal(got.numpy(), want)
    assert td.eligible_cells == d[f"t_{name}_eligible"].tolist()
    it = iter(td)
    for block, s, q, ok, nwarn in G.episodes(d, name):
        task = next(it)
        assert task.block_id == block
        np.testing.assert_array_equal(task.support["idx"].numpy(), s)
        np.testing.assert_array_equal(task.query["idx"].numpy(), q)
        assert int(task.metrics["image_disjoint_ok"]) == ok and len(task.warnings) == nwarn
        assert not np.isin(s, q).any()


def test_image_cap_greedy_equivalence():
    """The vectorised per-image cap equals the reference's greedy loop on random draws."""
    from adaptive_city_nerf_amd.data import TaskDataset
    g = np.random.default_rng(0)
    for trial in range(20):
        n = int(g.integers(1, 400))
        img = g.integers(0, int(g.integers(1, 9)), n)
        t = type("T", (), {})()
        t._img_indices = torch.from_numpy(img.astype(np.int32))
        t._rays, t._rgbs = torch.zeros(n, 8), torch.zeros(n, 3)
        cap = float(g.uniform(0.05, 1.0))
        td = TaskDataset(t, 0, image_cap=cap, min_rays_cell=1, region_bounds=((0, 0, 0), (1, 1, 1)), cells=(1, 1, 1),
                         bins=[torch.arange(n)], seed=trial)
        target = int(g.integers(1, n + 1))
        images = torch.unique(torch.from_numpy(img))
        state = td.rng.get_state()
        got = td._sample_split_from_images(0, target, images)
        td.rng.set_state(state)
        pool_idx, pool_img = td._cell_flat_idx[0], td._cell_flat_img[0]
        need = min(target, n)
        order = torch.randperm(n, generator=td.rng)
        capn = max(1, int(np.ceil(cap * need)))
        picked, counts = [], {}
        for pos in order.tolist():
            k = int(pool_img[pos])
            if counts.get(k, 0) >= capn:
                continue
            picked.append(pos)
            counts[k] = counts.get(k, 0) + 1
            if len(picked) >= need:
                break
        np.testing.assert_array_equal(got.numpy(), pool_idx[torch.tensor(picked, dtype=torch.long)].numpy())


def test_metadata_layout_and_masks(tmp_path):
    """get_image_metadata over the fixture written as a COLMAP-converted layout: indices over the sorted
    union of metadata files, scaled size/intrinsics, PNG load without resize, zipped mask + nearest
    resize (image_metadata.py:98-123)."""
    from adaptive_city_nerf_amd.data import get_image_metadata, discover_cluster_cells
    d = G.load("data_tasks")
    mdir = G.write_data_scene(tmp_path, d, 2)
    train, val = get_image_metadata(str(tmp_path), 0.125, mdir)
    items = [m for m in train if m is not None]
    assert val == [] and [m.image_index for m in items] == d["image_index"].tolist()
    for i, md in enumerate(items):
        assert (md.H, md.W) == tuple(int(v) for v in d["HW"])
        np.testing.assert_array_equal(md.intrinsics.numpy(), d["intrinsics"][i])
        np.testing.assert_array_equal(md.load_image().numpy(), d["images"][i])
        np.testing.assert_array_equal(md.load_mask().numpy(), D.mask_resize(G.data_masks(d, 2)[i], md.H, md.W))
    assert discover_cluster_cells(tmp_path / "masks" / "fixture") == 1
