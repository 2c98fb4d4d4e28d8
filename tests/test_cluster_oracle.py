"""Cluster creation on the CPU: pin oracle/cluster_ref.py + cluster_oracle.c
against scripts/create_clusters.py run on the CPU (tests/golden/clusters.npz, make_golden.py
gen_clusters), check the product's host logic (centroids, global box, final boxes, argument parsing)
and the cross-rank box reduction over gloo with world size 2.

Masks and indices are compared exactly; ray tables by SHA-256 of the reference's bytes.
"""
import hashlib
import json
import os
import socket
from pathlib import Path

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import goldens as G
from oracle import cluster_ref as CR

ROUTE_CASES = {"c2d_bm105": (0, "cent_grid22_2d", True, 1.05, 48),
               "c2d_strict": (7, "cent_grid42_2d", True, 1.0, 32),
               "c3d_bm110": (5, "cent_grid222_3d", False, 1.1, 40)}


def _cams(d):
    return torch.from_numpy(d["meta_c2w"])[..., :3, 3]


def test_centroids_match_reference():
    from adaptive_city_nerf_amd import clusters as CL
    d = G.load("clusters")
    cams = _cams(d)
    w = torch.tensor((d["meta_HW"][:, 0] * d["meta_HW"][:, 1]).astype(np.float32))
    for impl_grid, impl_km in ((CR.grid_centroids, CR.kmeans), (CL._grid_centroids, CL._run_kmeans)):
        np.testing.assert_array_equal(impl_grid(cams, 1, 2, 2, True).numpy(), d["cent_grid22_2d"])
        np.testing.assert_array_equal(impl_grid(cams, 1, 4, 2, True).numpy(), d["cent_grid42_2d"])
        np.testing.assert_array_equal(impl_grid(cams, 2, 2, 2, False).numpy(), d["cent_grid222_3d"])
        np.testing.assert_array_equal(impl_km(cams[:, 1:], 4, 50, "kmeans++", 0, None).numpy(), d["cent_km4_pp"])
        np.testing.assert_array_equal(impl_km(cams[:, 1:], 4, 50, "kmeans++", 0, w).numpy(), d["cent_km4_pp_w"])
        np.testing.assert_array_equal(impl_km(cams, 3, 20, "random", 5, None).numpy(), d["cent_km3_rand_3d"])


@pytest.mark.parametrize("name", list(ROUTE_CASES))
def test_oracle_routing_matches_reference(name):
    """compute_voronoi_orig (the reference's CPU path) on an image at 1/16 resolution: rays hash to the
    reference's bytes and every ray's centroid set is identical."""
    d = G.load("clusters")
    idx, cset, c2d, bm, S = ROUTE_CASES[name]
    H, W, fx, fy, cx, cy = d[f"route_{name}_hw_intr"]
    rays, valid = CR.cluster_rays(int(H), int(W), fx, fy, cx, cy, True, d["meta_c2w"][idx], d["route_gbox"])
    assert hashlib.sha256(rays.tobytes()).hexdigest() == str(d[f"route_{name}_rays_sha"])
    np.testing.assert_array_equal(valid, d[f"route_{name}_valid"])
    C = d[cset].shape[0]
    bits, _ = CR.voronoi(rays, S, d[cset], c2d, bm, orig=True)
    m = CR.bits_to_mask(bits, C)
    ref = np.unpackbits(d[f"route_{name}_mask"])[: m.size].reshape(m.shape).astype(bool)
    np.testing.assert_array_equal(m, ref)


def write_main_dataset(root: Path, d: dict, scale: float = 1.0 / 32.0) -> None:
    """The 4-image dataset gen_clusters ran main() on (coordinates + scaled metadata, no images)."""
    torch.save({"pose_scale_factor": float(d["pose_scale"]), "origin_drb": torch.from_numpy(d["origin_drb"]),
                "altitude_range_enu": torch.from_numpy(d["altitude_range_enu"])}, root / "coordinates.pt")
    for sp_stem in d["main_stems"]:
        split, stem = str(sp_stem).split("/")
        i = [k for k in range(len(d["meta_stem"])) if str(d["meta_stem"][k]) == stem
             and str(d["meta_split"][k]) == split][0]
        (root / split / "metadata").mkdir(parents=True, exist_ok=True)
        H, W = [int(v) for v in d["meta_HW"][i]]
        torch.save({"c2w": torch.from_numpy(d["meta_c2w"][i]), "H": int(H * scale), "W": int(W * scale),
                    "intrinsics": torch.from_numpy(d["meta_intr"][i]) * scale}, root / split / "metadata" / f"{stem}.pt")


MAIN_CASES = ("grid_orig", "kmeans_near_far", "grid3d")


def main_namespace(root: Path, case: str, orig: bool = True):
    from adaptive_city_nerf_amd import clusters as CL
    prm = json.loads(str(G.load("clusters")[f"main_{case}_params_json"]))
    argv = ["--data_path", str(root), "--output", case, "--centroid_mode", prm["centroid_mode"],
            "--boundary_margin", str(prm["boundary_margin"]), "--ray_samples", str(prm["ray_samples"]),
            "--center_pixels", "--scene_scale", "1.1", "--ray_chunk_size", "8192", "--sample_chunk_size", str(1 << 20)]
    argv += ["--grid_dim"] + [str(v) for v in ([2, 2] if prm["cluster_2d"] else [2, 1, 2])]
    if prm["cluster_2d"]:
        argv.append("--cluster_2d")
    n, f = prm["near_far_override_m"]
    if n is not None:
        argv += ["--near", str(n)]
    if f is not None:
        argv += ["--far", str(f)]
    if case == "kmeans_near_far":
        argv += ["--kmeans_weight_by_pixels", "--box_margin", "3.0"]
    if orig:
        argv.append("--orig")
    return CL.parse_args(argv)


@pytest.mark.parametrize("case", MAIN_CASES)
def test_main_glue_with_oracle_matches_reference(case, tmp_path):
    """main()'s host glue (argument parsing, global box, centroids, near/far override in metres, final
    boxes with empty experts + dilation + altitude band) from the product module, the per-image routing
    from the oracle: params, boxes and every mask equal the reference's end-to-end CPU run."""
    from adaptive_city_nerf_amd import clusters as CL
    d = G.load("clusters")
    write_main_dataset(tmp_path, d)
    h = main_namespace(tmp_path, case)
    coord = torch.load(tmp_path / "coordinates.pt", weights_only=True)
    box, ps = CL.global_scene_box(coord, h.scene_scale, h.altitude_range, h.altitude_pad)
    np.testing.assert_array_equal(box.aabb.numpy(), d[f"main_{case}_aabb_global"])
    metas = CL._meta_list(tmp_path, "train") + CL._meta_list(tmp_path, "val")
    cents, _ = CL.make_centroids(h, metas)
    np.testing.assert_array_equal(cents.numpy(), d[f"main_{case}_centroids"])
    nfo = (h.near / ps if h.near is not None else None, h.far / ps if h.far is not None else None)
    C = cents.shape[0]
    masks = []
    for p in CL._meta_list(tmp_path, "train") + CL._meta_list(tmp_path, "val"):
        md = torch.load(p, weights_only=True)
        fx, fy, cx, cy = [float(v) for v in md["intrinsics"]]
        rays, valid = CR.cluster_rays(md["H"], md["W"], fx, fy, cx, cy, True, md["c2w"].numpy(), box.aabb.numpy(), nfo)
        bits, _ = CR.voronoi(rays, h.ray_samples, cents.numpy(), h.cluster_2d, h.boundary_margin, orig=True)
        m = CR.bits_to_mask(bits, C) & valid[:, None]
        masks += [np.packbits(m[:, c]) for c in range(C)]
    np.testing.assert_array_equal(np.stack(masks), d[f"main_{case}_masks"])
    mins = torch.full((C, 3), float("inf"))
    maxs = torch.full((C, 3), float("-inf"))
    mn, mx = CL.final_boxes(mins, maxs, torch.zeros(C, dtype=torch.int64), cents, box.aabb, h.box_margin, ps)
    np.testing.assert_array_equal(mn.numpy(), d[f"main_{case}_mins"])
    np.testing.assert_array_equal(mx.numpy(), d[f"main_{case}_maxs"])
    np.testing.assert_array_equal(d[f"main_{case}_counts"], np.zeros(C, np.int64))


def test_final_boxes_product_equals_oracle():
    """Non-empty experts (the GPU path streams real boxes): product and oracle restatements agree,
    including NaN experts, clamping, dilation and the altitude band."""
    from adaptive_city_nerf_amd import clusters as CL
    g = torch.Generator().manual_seed(3)
    aabb = torch.tensor([[-0.05, -1.1, -1.1], [0.5, 1.1, 1.1]])
    mins = torch.rand(6, 3, generator=g) * 2.6 - 1.4
    maxs = mins + torch.rand(6, 3, generator=g)
    cnts = torch.tensor([5, 0, 7, 0, 3, 9])
    cents = torch.rand(6, 3, generator=g) * 3 - 1.5
    nanf = torch.tensor([0, 0, 0, 0, 1, 0], dtype=torch.int32)
    for margin in (0.0, 2.5):
        m1, M1 = CR.final_boxes(mins, maxs, cnts, cents, aabb, margin, 227.4, nan_flag=nanf)
        a, b = mins.clone(), maxs.clone()
        a[4] = float("nan")
        b[4] = float("nan")
        m2, M2 = CL.final_boxes(a, b, cnts, cents, aabb, margin, 227.4)
        np.testing.assert_array_equal(m1.numpy(), m2.numpy())
        np.testing.assert_array_equal(M1.numpy(), M2.numpy())


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _reduce_worker(rank, world, port, parts, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from adaptive_city_nerf_amd import clusters as CL
    mins, maxs, cnts, nan = [t.clone() for t in parts[rank]]
    mins, maxs, cnts = CL.reduce_boxes(mins, maxs, cnts, nan)
    q.put((rank, mins.numpy(), maxs.numpy(), cnts.numpy()))
    dist.destroy_process_group()


def test_box_reduction_two_ranks_gloo():
    """Rank-strided images: each rank streams its own boxes; MIN/MAX/SUM all-reduces (+ NaN flag) give
    the boxes a single process streaming every image gets (oracle on the CPU as the per-rank router)."""
    d = G.load("clusters")
    cents = d["cent_grid22_2d"]
    aabb = d["route_gbox"]
    parts, allrays = [], []
    for rank in range(2):
        st = (np.full((4, 3), np.inf, np.float32), np.full((4, 3), -np.inf, np.float32), np.zeros(4, np.int64),
              np.zeros(4, np.int32))
        for i in range(rank, 6, 2):
            H, W = [int(v) // 32 for v in d["meta_HW"][i]]
            fx, fy, cx, cy = [float(v) / 32 for v in d["meta_intr"][i]]
            rays, _ = CR.cluster_rays(H, W, fx, fy, cx, cy, True, d["meta_c2w"][i], aabb)
            allrays.append(rays)
            CR.voronoi(rays, 16, cents, True, 1.1, update=True, state=st)
        parts.append([torch.from_numpy(a) for a in st])
    single = (np.full((4, 3), np.inf, np.float32), np.full((4, 3), -np.inf, np.float32), np.zeros(4, np.int64),
              np.zeros(4, np.int32))
    for rays in allrays:
        CR.voronoi(rays, 16, cents, True, 1.1, update=True, state=single)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_reduce_worker, args=(r, 2, port, parts, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(2)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for _, mn, mx, cn in res:
        np.testing.assert_array_equal(mn, single[0])
        np.testing.assert_array_equal(mx, single[1])
        np.testing.assert_array_equal(cn, single[2])
    assert single[2].sum() > 0
