"""GPU parity of cluster creation: the routing kernel acn_voronoi_route against
the pinned oracle (oracle/cluster_oracle.c) bit for bit, main() end to end against the reference's
own CPU run (tests/golden/clusters.npz), and a full-scale run over the example dataset's 249 cameras
against the scene boxes / masks the reference produced on its GPU (shipped with the dataset)."""
import json
import zipfile

import numpy as np
import pytest
import torch

import goldens as G
from oracle import cluster_ref as CR
from test_cluster_oracle import MAIN_CASES, main_namespace, write_main_dataset

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _rays_small(d, idx=0, div=16, extra=True):
    H, W = [int(v) // div for v in d["meta_HW"][idx]]
    fx, fy, cx, cy = [float(v) / div for v in d["meta_intr"][idx]]
    rays, _ = CR.cluster_rays(H, W, fx, fy, cx, cy, True, d["meta_c2w"][idx], d["route_gbox"])
    if extra:  # invalid rays (inf near/far -> NaN samples), a degenerate segment, axis-parallel rays
        e = np.tile(rays[:64].copy(), (1, 1))
        e[:16, 6:8] = np.inf
        e[16:32, 7] = e[16:32, 6]
        e[32:48, 3:6] = np.array([0.0, 0.0, 1.0], np.float32)
        e[48:64, 3:6] = np.array([1.0, 0.0, 0.0], np.float32)
        rays = np.concatenate([rays, e], 0)
    return np.ascontiguousarray(rays, np.float32)


def _cents(n, three_d, seed):
    g = np.random.default_rng(seed)
    c = g.uniform(-0.9, 0.9, (n, 3)).astype(np.float32)
    if not three_d:
        c[:, 0] = 0.0
    return c


@pytest.mark.parametrize("mode", ["strict", "overlap", "orig"])
@pytest.mark.parametrize("c2d", [True, False])
@pytest.mark.parametrize("C,S", [(1, 8), (4, 64), (8, 17), (12, 2), (40, 5)])
def test_route_kernel_matches_oracle(mode, c2d, C, S):
    from adaptive_city_nerf_amd import clusters as CL
    d = G.load("clusters")
    rays = _rays_small(d, idx=(C * 7) % 249)
    cents = _cents(C, not c2d, C + S)
    bm = {"strict": 1.0, "overlap": 1.07, "orig": 1.05}[mode]
    orig = mode == "orig"
    wb, (wmin, wmax, wcnt, wnan) = CR.voronoi(rays, S, cents, c2d, bm, orig=orig, update=not orig)
    mins = torch.full((C, 3), float("inf"), device=DEV)
    maxs = torch.full((C, 3), float("-inf"), device=DEV)
    cnts = torch.zeros(C, dtype=torch.int64, device=DEV)
    nan = torch.zeros(C, dtype=torch.int32, device=DEV)
    bits = CL.voronoi_route(torch.from_numpy(rays).to(DEV), S, torch.from_numpy(cents), c2d, bm, orig=orig,
                            update_aabbs=not orig, mins_out=mins, maxs_out=maxs, counts_out=cnts, nan_out=nan)
    np.testing.assert_array_equal(bits.cpu().numpy().view(np.uint64), wb)
    if not orig:
        np.testing.assert_array_equal(cnts.cpu().numpy(), wcnt)
        np.testing.assert_array_equal(nan.cpu().numpy(), wnan)
        np.testing.assert_array_equal(mins.cpu().numpy(), wmin)
        np.testing.assert_array_equal(maxs.cpu().numpy(), wmax)
        if mode == "strict":
            assert wnan[0] == 1  # the invalid rays' NaN samples go to centroid 0, as torch.argmin does


def test_image_rays_match_oracle():
    from adaptive_city_nerf_amd import clusters as CL
    from adaptive_city_nerf_amd.scene_box import SceneBox
    d = G.load("clusters")
    box = SceneBox(aabb=torch.from_numpy(d["route_gbox"]).to(DEV))
    for idx, nfo in ((3, (None, None)), (200, (0.004, 0.8))):
        H, W = [int(v) // 8 for v in d["meta_HW"][idx]]
        intr = torch.from_numpy(d["meta_intr"][idx]) / 8
        md = {"H": H, "W": W, "intrinsics": intr, "c2w": torch.from_numpy(d["meta_c2w"][idx])}
        rays, valid = CL.image_rays(md, True, box, nfo, DEV)
        fx, fy, cx, cy = [float(v) for v in intr]
        wr, wv = CR.cluster_rays(H, W, fx, fy, cx, cy, True, d["meta_c2w"][idx], d["route_gbox"], nfo)
        np.testing.assert_array_equal(rays.cpu().numpy(), wr)
        np.testing.assert_array_equal(valid.cpu().numpy(), wv)


def _read_masks(od, stems, C):
    out = []
    for sp_stem in stems:
        stem = str(sp_stem).split("/")[1]
        for c in range(C):
            with zipfile.ZipFile(od / str(c) / f"{stem}.pt") as zf, zf.open(zf.namelist()[0]) as f:
                out.append(np.packbits(torch.load(f, weights_only=True).numpy().reshape(-1)))
    return np.stack(out)


@pytest.mark.parametrize("case", MAIN_CASES)
def test_main_end_to_end_matches_reference(case, tmp_path):
    """create_clusters main (--orig, the reference's CPU path) on the fixture dataset: params.pt,
    scene_boxes.pt and every zipped mask equal the reference's files."""
    from adaptive_city_nerf_amd import clusters as CL
    d = G.load("clusters")
    write_main_dataset(tmp_path, d)
    saved = CL.main(main_namespace(tmp_path, case))
    od = tmp_path / "masks" / case
    C = saved["centroids"].shape[0]
    np.testing.assert_array_equal(_read_masks(od, d["main_stems"], C), d[f"main_{case}_masks"])
    boxes = torch.load(od / "scene_boxes.pt", weights_only=True)
    for key in ("mins", "maxs", "counts", "centroids", "aabb_global"):
        np.testing.assert_array_equal(boxes[key].numpy(), d[f"main_{case}_{key}"])
    params = torch.load(od / "params.pt", weights_only=True)
    ref = json.loads(str(d[f"main_{case}_params_json"]))
    got = {k: (list(v) if isinstance(v, tuple) else v) for k, v in params.items() if not isinstance(v, torch.Tensor)}
    assert got == ref
    assert (od / "scene_boxes.txt").exists()


def test_main_opt_streams_boxes_like_oracle(tmp_path):
    """Default (opt) mode: masks and the streamed per-expert boxes / counts equal the oracle's."""
    from adaptive_city_nerf_amd import clusters as CL
    d = G.load("clusters")
    write_main_dataset(tmp_path, d)
    h = main_namespace(tmp_path, "grid_orig", orig=False)
    saved = CL.main(h)
    cents = saved["centroids"].numpy()
    C = cents.shape[0]
    coord = torch.load(tmp_path / "coordinates.pt", weights_only=True)
    box, ps = CL.global_scene_box(coord, h.scene_scale, h.altitude_range, h.altitude_pad)
    st = (np.full((C, 3), np.inf, np.float32), np.full((C, 3), -np.inf, np.float32), np.zeros(C, np.int64),
          np.zeros(C, np.int32))
    masks = []
    for p in CL._meta_list(tmp_path, "train") + CL._meta_list(tmp_path, "val"):
        md = torch.load(p, weights_only=True)
        fx, fy, cx, cy = [float(v) for v in md["intrinsics"]]
        rays, valid = CR.cluster_rays(md["H"], md["W"], fx, fy, cx, cy, True, md["c2w"].numpy(), box.aabb.numpy())
        bits, _ = CR.voronoi(rays, h.ray_samples, cents, True, h.boundary_margin, update=True, state=st)
        m = CR.bits_to_mask(bits, C) & valid[:, None]
        masks += [np.packbits(m[:, c]) for c in range(C)]
    np.testing.assert_array_equal(_read_masks(tmp_path / "masks" / "grid_orig", d["main_stems"], C), np.stack(masks))
    mn, mx = CR.final_boxes(st[0], st[1], st[2], cents, box.aabb, 0.0, ps, nan_flag=st[3])
    np.testing.assert_array_equal(saved["mins"].numpy(), mn.numpy())
    np.testing.assert_array_equal(saved["maxs"].numpy(), mx.numpy())
    np.testing.assert_array_equal(saved["counts"].numpy(), st[2])
    assert st[2].min() > 0


def test_full_dataset_against_shipped_reference_outputs():
    """All 249 cameras at full resolution (1536 x 2048, 256 samples, g22 grid, margin 1.1, centred
    pixels): the streamed per-expert boxes and sample counts against scene_boxes.pt that the reference
    produced on its GPU, and two images' masks against its zipped masks.  The reference's GPU path runs
    its direction / distance GEMMs in TF32 on Ampere-class GPUs (create_clusters.py:87-89) while this
    path is exact fp32, yet the boxes come out bit-identical and both images' masks identical; the
    sample counts (5.4e10-5.7e10 per expert) differ by a few tens of boundary samples (measured:
    +30, -24, -34, +36), bounded here at 1e-8 relative."""
    from adaptive_city_nerf_amd import clusters as CL
    from adaptive_city_nerf_amd.scene_box import SceneBox
    d = G.load("clusters")
    tag = "ship_g22_grid_bm110_ss11"
    prm = json.loads(str(d[f"{tag}_params_json"]))
    cents = torch.from_numpy(d[f"{tag}_centroids"])
    aabb = torch.from_numpy(d[f"{tag}_aabb_global"])
    box = SceneBox(aabb=aabb.to(DEV))
    C = cents.shape[0]
    mins = torch.full((C, 3), float("inf"), device=DEV)
    maxs = torch.full((C, 3), float("-inf"), device=DEV)
    cnts = torch.zeros(C, dtype=torch.int64, device=DEV)
    nan = torch.zeros(C, dtype=torch.int32, device=DEV)
    agree = {}
    for i in range(len(d["meta_stem"])):
        H, W = [int(v) for v in d["meta_HW"][i]]
        md = {"H": H, "W": W, "intrinsics": torch.from_numpy(d["meta_intr"][i]),
              "c2w": torch.from_numpy(d["meta_c2w"][i])}
        rays, valid = CL.image_rays(md, True, box, (None, None), DEV)
        bits = CL.voronoi_route(rays, prm["ray_samples"], cents, True, prm["boundary_margin"], update_aabbs=True,
                                mins_out=mins, maxs_out=maxs, counts_out=cnts, nan_out=nan)
        stem = str(d["meta_stem"][i])
        if f"ship_mask_{stem}_0" in d:
            m = (CL.bits_to_masks(bits, C) & valid.view(-1, 1)).cpu().numpy()
            for c in range(C):
                ref = np.unpackbits(d[f"ship_mask_{stem}_{c}"])[: H * W].astype(bool)
                agree[(stem, c)] = float((m[:, c] == ref).mean())
    torch.cuda.synchronize()
    mins, maxs, cnts = CL.reduce_boxes(mins, maxs, cnts, nan)
    mn, mx = CL.final_boxes(mins, maxs, cnts, cents.to(DEV), aabb.to(DEV), 0.0, 1.0)
    print("mask agreement", agree)
    print("mins", mn.cpu().numpy().tolist(), "ref", d[f"{tag}_mins"].tolist())
    print("maxs", mx.cpu().numpy().tolist(), "ref", d[f"{tag}_maxs"].tolist())
    print("counts", cnts.cpu().numpy().tolist(), "ref", d[f"{tag}_counts"].tolist())
    assert len(agree) == 2 * C and min(agree.values()) == 1.0
    np.testing.assert_array_equal(mn.cpu().numpy(), d[f"{tag}_mins"])
    np.testing.assert_array_equal(mx.cpu().numpy(), d[f"{tag}_maxs"])
    np.testing.assert_allclose(cnts.cpu().numpy(), d[f"{tag}_counts"], rtol=1e-8)
