#!/usr/bin/env python3
"""bench.py -- BASELINE.json metric "ray-samples/sec + PSNR" on BASELINE config C2.

Workload (one "step"): render_rays() of 4096 rays x 256 stratified samples through ONE Instant-NGP
expert (L=16 hash grid, T=2^20, F=2; sigma 2x64; colour 2x64; SH-4; background MLP), eval mode,
fp32 -- a single fused HIP launch of the product API (adaptive_city_nerf_amd.render_rays).
Inputs are resident in HBM before timing: rays from validation camera 0 of the reference's
example scene at downscale 0.25 (geometry from tests/golden/scene_drz_example.json), 4096 valid
rays drawn without replacement (seed 1234 + rank); hash table formula-filled U(-0.5, 0.5)
(synthetic.py); MLP weights default nn.Linear init under torch.manual_seed(0).

Multi-GPU (torch.distributed.run, one process per GPU): rays are independent, so every rank renders
its own 4096 x 256 batch (weak scaling, no collective in the data path); barrier + synchronize
bracket the K timed steps and the max over ranks is reported.

Other BASELINE configs (``--workload``):
  c3  2x2 Voronoi grid -> 4 experts (soft routing, boundary_margin 1.05); a global batch of
      world x 4096 rays x 256 samples is sharded by owning expert (parallel.expert_sorted_plan),
      each rank renders its 4096 rays and the rendered rays are all-gathered over RCCL (weak).
  c4  4x2 grid -> 8 experts (synthetic layout, synthetic.grid_layout), one 800x800 frame x 256
      samples: rays generated on device, sharded by expert, rendered, all-gathered, PSNR
      all-reduced (parallel.render_image_sharded) -- strong scaling.
  c5  online adaptation (runtime_adapt.py:286-309): the routed 8-expert container (no active_module)
      on batches of 1000 rays x 96 samples from a 249-camera stream: training render -> MSE ->
      backward -> clip_grad_norm_ + Adam over every expert hit.  1 GPU: routed_train.RoutedAdaptStep
      replayed as one HIP graph; N GPUs: experts distributed (expert_parallel.py, all-to-all of
      per-sample records), each rank streaming its own batches (weak).  metric value = trained
      ray-samples/s (fwd+bwd+update); also the val PSNR before / after the adaptation.
  c5a placement variant: rank r adapts expert r alone (active_module), no collective.

Also reported: roofline of the fused render kernel (HIP events bracketing exactly that launch on
its stream), and on rank 0 at N=1 a CPU baseline: the C oracle (oracle/, a fixture-pinned port of
the reference CPU path) rendering the same batch on the host cores, whose output also gives the
PSNR of the GPU render against the CPU path.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path
from typing import Optional

import numpy as np
import torch
import torch.distributed as dist

REPO = Path(__file__).resolve().parent
sys.path.insert(0, str(REPO))

FLOP_PER_SAMPLE = 26880          # MLP MACs x 2: 32*64+64*64+64+64*15+31*64+64*64+64*3 = 13,440
BYTES_PER_SAMPLE = 1024.2        # algorithmic hash-table reads + amortised ray I/O
FP32_MFMA_PEAK_TFLOPS = 157.3    # MI355X_MICROARCH.md: FP32 matrix = vector peak (spec)
HBM_PEAK_GBS = 8000.0
ATOMIC_REQ_PEAK = 1.3e12 / 64   # memory-side float-atomic requests/s (MI355X_MICROARCH.md 'Global float atomics')


def build_model(device, n_experts=1, seed=0, table_seed=100, table_scale=0.5, fill=None, occ_conf=None,
                expert_box="own"):
    from adaptive_city_nerf_amd import MetaContainer, SceneBox
    from adaptive_city_nerf_amd.synthetic import formula_table, grid_layout
    scene = json.loads((REPO / "tests" / "golden" / "scene_drz_example.json").read_text())
    if n_experts in (1, 4):
        sc = scene["masks"]["g11_grid_bm110_ss11" if n_experts == 1 else "g22_grid_bm110_ss11"]
    elif n_experts == 8:
        sc = grid_layout(4, 2, scene)
    else:
        raise ValueError("n_experts must be 1 (g11), 4 (g22) or 8 (synthetic g42)")
    K = len(sc["centroids"])
    gbox = SceneBox(aabb=torch.tensor(sc["aabb_global"], dtype=torch.float32))
    boxes = [SceneBox(aabb=torch.tensor([sc["mins"][k], sc["maxs"][k]], dtype=torch.float32)) for k in range(K)]
    if expert_box == "global":      # diagnostic: every expert's encoder normalises by the whole-scene box
        boxes = [SceneBox(aabb=gbox.aabb.clone()) for _ in range(K)]
    torch.manual_seed(seed)
    m = MetaContainer(num_submodules=K, centroids=torch.tensor(sc["centroids"]), aabb=gbox.aabb,
                      nerf_variant="instant", boundary_margin=min(max(1.0, 1.05), sc["boundary_margin"]),
                      cluster_2d=sc["cluster_2d"], use_bg_nerf=True, bg_hidden=32,
                      occ_conf=occ_conf or {"use_occ": False},
                      expert_box_list=boxes, hidden=64, sigma_depth=2, color_depth=2, dir_encoding="spherical",
                      color_hidden=64, use_sigmoid_rgb=True,
                      hash_enc_conf={"levels": 16, "features_per_level": 2, "log2_hashmap_size": 20,
                                     "max_res": 4096, "min_res": 16, "interpolation": "Linear"})
    with torch.no_grad():
        for k, sub in enumerate(m.submodules):
            if fill is None or k in fill:
                sub.xyz_encoder.hash_table.copy_(torch.from_numpy(formula_table(16, 20, 2, table_seed + k, table_scale)))
    return m.to(device).eval(), gbox, scene, sc


def frame_camera(scene, H=None, W=None, ds=0.25):
    """Validation camera 0: at downscale ds, or with intrinsics rescaled to an H x W frame
    centred at (W/2, H/2) (800x800, cx = cy = 400)."""
    cam = scene["val_cam0"]
    intr = torch.tensor(cam["intrinsics"], dtype=torch.float32)
    if H is None:
        return int(round(cam["H"] * ds)), int(round(cam["W"] * ds)), (intr * ds).tolist(), torch.tensor(cam["c2w"])
    s = min(H / cam["H"], W / cam["W"])
    return H, W, [float(intr[0] * s), float(intr[1] * s), W / 2.0, H / 2.0], torch.tensor(cam["c2w"])


def make_rays(scene, gbox, device, n_rays, seed, pixel_order=False):
    from adaptive_city_nerf_amd import ops
    H, W, intr, c2w = frame_camera(scene)
    psf = scene["pose_scale_factor"]
    rays, valid = ops.get_rays_image(H, W, *intr, c2w, gbox.aabb, device,
                                     near_far_override=(0.0 / psf, 100000 / psf))
    vi = torch.nonzero(valid).squeeze(1).cpu()
    g = torch.Generator().manual_seed(seed)
    sel = vi[torch.randperm(vi.numel(), generator=g)[:n_rays]]
    if pixel_order:
        sel = torch.sort(sel).values
    return rays[sel.to(device)].contiguous()


def make_rays_multi(gbox, device, n_rays, seed, ds=0.125, cams=None):
    """Rays of random valid pixels over the example dataset's 249 cameras (train + val poses and
    intrinsics, tests/golden/clusters.npz from the reference's metadata) at downscale ``ds`` -- the
    stream a runtime_adapt data loader draws from a whole continual batch (every expert is reached)."""
    from adaptive_city_nerf_amd import ops
    z = np.load(REPO / "tests" / "golden" / "clusters.npz", allow_pickle=False)
    c2ws, intrs, hws = z["meta_c2w"], z["meta_intr"], z["meta_HW"]
    psf = float(z["pose_scale"])
    g = torch.Generator().manual_seed(seed)
    idx = torch.randperm(len(c2ws), generator=g).tolist() if cams is None else list(cams)
    out, total = [], 0
    for i in idx:
        H, W = int(round(hws[i][0] * ds)), int(round(hws[i][1] * ds))
        fx, fy, cx, cy = (float(v) * ds for v in intrs[i])
        rays, valid = ops.get_rays_image(H, W, fx, fy, cx, cy, torch.from_numpy(c2ws[i]), gbox.aabb, device,
                                         near_far_override=(0.0, 100000 / psf))
        out.append(rays[valid])
        total += out[-1].shape[0]
        if total >= 4 * n_rays and len(out) >= 16:
            break
    allr = torch.cat(out)
    sel = torch.randperm(allr.shape[0], generator=g)[:n_rays].to(device)
    return allr[sel].contiguous()


def cpu_baseline(model, sc, rays, S, gpu_rgb, min_seconds):
    """C oracle on the host cores over the same batch, repeated until >= min_seconds."""
    from oracle import oracle as O
    experts = []
    for sub in model.submodules:
        w = {n: p.detach().cpu().numpy() for n, p in sub.meta_named_parameters()}
        experts.append(O.Expert(w, sub.xyz_encoder.hash_table.detach().cpu().numpy(),
                                np.array(sub.xyz_encoder._res_host, np.int32), sub.scene_box.min.cpu().numpy(),
                                sub.aabb_extent.cpu().numpy()))
    bg = {f"bg_mlp.{k}": v.detach().cpu().numpy() for k, v in model.bg_mlp.state_dict().items()}
    r = rays.cpu().numpy()
    cores = O.max_threads()
    reps, t0 = 0, time.perf_counter()
    while True:
        orgb, _, _, _ = O.render_stratified(r, S, experts, np.array(sc["centroids"], np.float32),
                                            bm=model.boundary_margin, bg_mlp=bg, want_weights=False)
        reps += 1
        if time.perf_counter() - t0 >= min_seconds:
            break
    dt = time.perf_counter() - t0
    mse = float(np.mean((gpu_rgb.astype(np.float64) - orgb.astype(np.float64)) ** 2))
    psnr = float("inf") if mse == 0 else -10.0 * np.log10(mse)
    # one thread (SURVEY §8(d) "also report one-thread"): a bounded prefix of the same batch
    n1 = min(r.shape[0], 256)
    O.set_threads(1)
    try:
        reps1, t1 = 0, time.perf_counter()
        while True:
            O.render_stratified(r[:n1], S, experts, np.array(sc["centroids"], np.float32), bm=model.boundary_margin,
                                bg_mlp=bg, want_weights=False)
            reps1 += 1
            if time.perf_counter() - t1 >= min(5.0, min_seconds):
                break
        dt1 = time.perf_counter() - t1
    finally:
        O.set_threads(cores)
    single = {"value": n1 * S * reps1 / dt1, "unit": "ray-samples/s", "cores": 1,
              "sample": f"{reps1} x ({n1} rays x {S} samples), C oracle single thread, {dt1:.1f} s"}
    return {"value": r.shape[0] * S * reps / dt, "unit": "ray-samples/s", "cores": cores, "kind": "port",
            "sample": f"{reps} x ({r.shape[0]} rays x {S} samples) of the benchmark batch, C oracle "
                      f"(oracle/acn_oracle.c, OpenMP {cores} threads), {dt:.1f} s",
            "single_thread": single}, psnr, float(np.sqrt(mse)), float(np.max(np.abs(gpu_rgb - orgb)))


def cpu_baseline_train(model, sc, rays, rgbs, S, expert, min_seconds):
    """C5 CPU baseline: the CPU restatement of one runtime_adapt update (oracle/train_ref.py, pinned
    by the reference's training fixtures, incl. the K=8 routed container at 1000 x 96) on the host
    cores, same batch shape, repeated >= min_seconds.  expert=None: the routed container."""
    from oracle import oracle as O
    from oracle import train_ref as TR
    state = {k: v.detach().cpu() for k, v in model.state_dict().items()}
    K = len(model.submodules)
    m = TR.RefContainer(state, K, np.array(model.submodules[0].xyz_encoder._res_host), 20, sc["centroids"],
                        model.boundary_margin, sc["mins"], [s.aabb_extent.cpu().numpy() for s in model.submodules])
    lrs = {"encoding": 0.01, "sigma": 0.002, "color": 0.002, "background": 0.001}
    opt = torch.optim.Adam(m.param_groups(lrs), lr=1e-4)
    threads = O.max_threads()
    torch.set_num_threads(threads)
    r, g = rays.cpu(), rgbs.cpu()
    u = torch.rand(r.shape[0], S, generator=torch.Generator().manual_seed(3))
    reps, t0 = 0, time.perf_counter()
    while True:
        TR.adapt_step(m, opt, r, g, S, u, active_module=expert)
        reps += 1
        if time.perf_counter() - t0 >= min_seconds:
            break
    dt = time.perf_counter() - t0
    return {"value": r.shape[0] * S * reps / dt, "unit": "ray-samples/s", "cores": threads, "kind": "port",
            "sample": f"{reps} runtime_adapt updates of {r.shape[0]} rays x {S} samples through "
                      f"{'the routed ' + str(K) + '-expert container' if expert is None else 'expert ' + str(expert)} "
                      f"(oracle/train_ref.py: PyTorch CPU restatement, fixture-pinned; {threads} threads), "
                      f"{dt:.1f} s"}


def cpu_baseline_occ(model, rays, gpu_rgb, min_seconds):
    """Occupancy renderer on the host cores: oracle/occ_ref.render_expert_occ (C traversal + C field +
    numpy compositing) over the same rays and grid, repeated until >= min_seconds."""
    from oracle import occ_ref as R
    from oracle import oracle as O
    sub = model.submodules[0]
    w = {n: p.detach().cpu().numpy() for n, p in sub.meta_named_parameters()}
    e = O.Expert(w, sub.xyz_encoder.hash_table.detach().cpu().numpy(), np.array(sub.xyz_encoder._res_host, np.int32),
                 sub.scene_box.min.cpu().numpy(), sub.aabb_extent.cpu().numpy())
    b = sub.occ_grid.binaries.cpu().numpy()
    ab = sub.occ_grid.aabbs.cpu().numpy()
    r = rays.cpu().numpy()
    reps, n, t0 = 0, 0, time.perf_counter()
    while True:
        orgb, _, wts, _, smp = R.render_expert_occ(e, r, b, ab, sub.render_step_size, sub.cone_angle)
        reps += 1
        n += len(smp[1])
        if time.perf_counter() - t0 >= min_seconds:
            break
    dt = time.perf_counter() - t0
    mse = float(np.mean((gpu_rgb.astype(np.float64) - orgb.astype(np.float64)) ** 2))
    psnr = float("inf") if mse == 0 else -10.0 * np.log10(mse)
    cores = O.max_threads()
    return {"value": n / dt, "unit": "ray-samples/s", "cores": cores, "kind": "port",
            "sample": f"{reps} x {r.shape[0]} rays ({n // reps} marched samples) of the benchmark batch, "
                      f"oracle/occ_ref.py (C traversal and field with OpenMP {cores} threads, numpy compositing), "
                      f"{dt:.1f} s"}, psnr, float(np.sqrt(mse)), float(np.max(np.abs(gpu_rgb - orgb)))


def cpu_baseline_data(td, rays, gpu_bins, min_seconds):
    """_route_and_bin on the host cores: oracle/data_ref.route (float32 numpy restatement of the
    reference's torch CPU routing) + the reference's argsort binning, on a bounded prefix of the
    region's rays; its bins are checked against the GPU's for that prefix."""
    from oracle import data_ref as DR
    n = min(rays.shape[0], 1 << 19)
    r = rays[:n].cpu().numpy()
    aabb = td.aabb.numpy()
    reps, t0 = 0, time.perf_counter()
    while True:
        cid, flags = DR.route(r, aabb, td.cells, td.assignment_checkpoint, td.routing_policy)
        bins = DR.bins(cid, flags, int(np.prod(td.cells)))
        reps += 1
        if time.perf_counter() - t0 >= min_seconds:
            break
    dt = time.perf_counter() - t0
    full = [b.cpu().numpy() for b in gpu_bins]
    same = all(np.array_equal(np.sort(b[b < n]), np.sort(c)) for b, c in zip(full, bins))
    return {"value": reps * n / dt, "unit": "rays/s", "cores": 1, "kind": "port",
            "sample": f"{reps} x {n} rays (prefix of the region table), oracle/data_ref.py route+bins (numpy, "
                      f"single thread), {dt:.1f} s; per-cell membership equal to the GPU bins: {same}"}


def cpu_baseline_clusters(out, cents, S, min_seconds):
    """create_clusters routing on the host cores: oracle/cluster_ref.voronoi (C, one thread) over a
    bounded prefix of the same frame's rays; its bits are checked against the GPU's for that prefix."""
    from oracle import cluster_ref as CR
    bits, _, rays = out
    n = 1 << 14
    r = rays[:n].cpu().numpy()
    reps, t0 = 0, time.perf_counter()
    while True:
        got, _ = CR.voronoi(r, S, cents.numpy(), True, 1.1, update=True)
        reps += 1
        if time.perf_counter() - t0 >= min_seconds:
            break
    dt = time.perf_counter() - t0
    same = bool(np.array_equal(got, bits[:n].cpu().numpy().view(np.uint64)))
    return {"value": reps * n * S / dt, "unit": "ray-samples/s", "cores": 1, "kind": "port",
            "sample": f"{reps} x {n} rays x {S} samples of the benchmark frame, oracle/cluster_oracle.c "
                      f"(single thread), {dt:.1f} s; bits equal to the GPU's: {same}"}


def cpu_baseline_meta(model, sc, task_data, S, min_seconds):
    """Meta-training on the host cores: oracle/meta_ref.py (the fixture-pinned PyTorch CPU restatement
    of train_step) on a bounded sample: one region, one task cut to 500 support + 250 query rays, the
    configured inner steps; repeated until >= min_seconds; samples counted like the GPU line."""
    from oracle import meta_ref as MR
    from oracle import oracle as O
    from oracle import train_ref as TR
    state = {k: v.detach().cpu() for k, v in model.state_dict().items()}
    K = len(model.submodules)
    m = TR.RefContainer(state, K, np.array(model.submodules[0].xyz_encoder._res_host), 20, sc["centroids"],
                        model.boundary_margin, sc["mins"], [s.aabb_extent.cpu().numpy() for s in model.submodules])
    lrs = {"encoding": 0.01, "sigma": 0.002, "color": 0.002, "background": 0.001}
    opt = torch.optim.Adam(m.param_groups(lrs), lr=1e-4)
    threads = O.max_threads()
    torch.set_num_threads(threads)
    t = task_data[0][0]
    ns, nq, iters = 500, 250, 8
    task = {0: {"support": {k: v[:ns].cpu() for k, v in t["support"].items()},
                "query": {k: v[:nq].cpu() for k, v in t["query"].items()}}}
    g = torch.Generator().manual_seed(3)
    reps, t0 = 0, time.perf_counter()
    while True:
        us = iter([torch.rand(ns, S, generator=g) for _ in range(iters)] + [torch.rand(nq, S, generator=g)])
        MR.meta_step(m, opt, task, [0], S, us, "fomaml", 0.015, iters, 1e-4)
        reps += 1
        if time.perf_counter() - t0 >= min_seconds:
            break
    dt = time.perf_counter() - t0
    n = reps * (iters * ns + nq) * S
    return {"value": n / dt, "unit": "ray-samples/s", "cores": threads, "kind": "port",
            "sample": f"{reps} meta steps of 1 region x 1 task ({ns} support x {iters} inner + {nq} query rays, "
                      f"{S} samples; oracle/meta_ref.py PyTorch CPU restatement, {threads} threads), {dt:.1f} s"}


def hash_bwd_segments(routed) -> int:
    """Distinct 64-B segments (8 rows of 8 B) of the gradient tables one routed step's table scatter
    touches: the floor on memory-side atomic requests of any scatter-add of these contributions
    (MI355X_MICROARCH.md 'Global float atomics': one request per 64-B segment an atomic
    wave-instruction covers).  Same hash and corner set as hashgrid_bwd_pairs (encoders.hip)."""
    K = routed.K
    live = int(routed.seg[K])
    keep = routed.pidx[:live] >= 0
    x = routed.x01[:live][keep]
    pk = routed.pk[:live][keep].long()
    enc = routed.model.submodules[0].xyz_encoder
    log2T, mask = enc.log2_hashmap_size, (1 << enc.log2_hashmap_size) - 1
    P1, P2, U32 = 2654435761, 805459861, 0xFFFFFFFF
    keys = []
    for l, r in enumerate(enc._res_host):
        s = torch.floor(x * float(r)).long()
        for c in range(8):
            bx, by, bz = c >> 2, (c >> 1) & 1, c & 1
            h = (((s[:, 0] + bx) & U32) ^ (((s[:, 1] + by) * P1) & U32) ^ (((s[:, 2] + bz) * P2) & U32)) & mask
            keys.append((((pk * len(enc._res_host) + l) << log2T) | h) >> 3)
    return int(torch.unique(torch.cat(keys)).numel())


def load_traffic(name: str = "render", rnd: str = "r01"):
    """Committed per-launch HBM bytes of a workload's dominant kernel (profiles/pmc_<name>_<round>.json,
    from separate rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes: tools/pmc_kernel.sh + pmc_fold.py,
    tools/pmc_c5.sh)."""
    p = REPO / "profiles" / f"pmc_{name}_{rnd}.json"
    if p.exists():
        try:
            return json.loads(p.read_text())
        except Exception:
            return None
    return None


def render_traffic_profile(workload: str, S: int, layout: str):
    """Counter summary of the render line's dominant kernel (tools/pmc_r04.sh + tools/pmc_fold_r04.py: separate
    rocprofv3 --pmc passes, FETCH_SIZE doubled per the gfx950 correction of MI355X_MICROARCH.md 'HBM', plus
    WRITE_SIZE) -- round 6, the final render build (buffer-load gathers, depth tiles; C4 at S = 256 not profiled) -- or None
    when no profile of this exact configuration is committed."""
    name = {("c2", 256, "replicated"): "r06_pmc_c2_render.json",
            ("c3", 256, "replicated"): "r06_pmc_c3_render.json",
            ("c4", 96, "replicated"): "r06_pmc_c4s96_render.json"}.get((workload, S, layout))
    if name is None:
        return None
    p = REPO / "profiles" / name
    try:
        d = json.loads(p.read_text())
    except Exception:
        return None
    d["_source"] = f"profiles/{name}"
    return d


def load_gather_ceiling():
    """Committed gather-only ceiling of the render's hash access (tools/micro/hash_gather.py on the GPU box:
    profiles/r03_hash_gather_ceiling.json)."""
    p = REPO / "profiles" / "r03_hash_gather_ceiling.json"
    try:
        return json.loads(p.read_text())
    except Exception:
        return None


def free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_command(argv, n_gpus: int, port: int):
    """torch.distributed.run command that starts ``n_gpus`` ranks of this script with the same
    arguments (one process per GPU, rendezvous on 127.0.0.1)."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n_gpus}",
            "--master-addr=127.0.0.1", f"--master-port={port}", str(Path(__file__).resolve()), *argv]


def maybe_launch(argv, n_gpus: int) -> Optional[int]:
    """``bench.py --gpus N`` run directly (no WORLD_SIZE in the environment) with N > 1: start the N
    ranks as a child torch.distributed.run and return its exit code.  Runs before anything touches
    the GPU (the parent never initialises HIP, so nothing is re-exec'd from a GPU process)."""
    if n_gpus <= 1 or "WORLD_SIZE" in os.environ:
        return None
    import subprocess
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.run(launch_command(argv, n_gpus, free_port()), env=env).returncode


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=None,
                    help="timed steps (default 200 for the sub-millisecond c2 / c3 steps, whose fixed start-up "
                         "latency would otherwise weigh on a 20-step window; 20 for the others)")
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--workload", choices=["c2", "c3", "c4", "c5", "c5a", "occ", "meta", "data", "clusters"], default="c2")
    ap.add_argument("--rays", type=int, default=4096, help="rays per GPU (c2, c3)")
    ap.add_argument("--samples", type=int, default=256)
    ap.add_argument("--frame", type=int, default=800, help="frame side (c4)")
    ap.add_argument("--layout", choices=["replicated", "expert"], default="replicated",
                    help="c4: experts replicated + rays sharded by owning expert (all-gather of rendered rays), or "
                         "one expert per GPU (all-to-all of per-sample records, expert_parallel.py)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--opaque", type=float, default=0.0,
                    help="c2: add this to every expert's sigma_head bias (density x e^B): a synthetic opaque "
                         "scene on which early ray termination has rays to stop")
    ap.add_argument("--tau", type=float, default=0.0,
                    help="c2: early ray termination threshold on transmittance (wavefront scan; 0 = off, the "
                         "reference's behaviour); the line then reports the RGB error against tau = 0")
    ap.add_argument("--cpu-rays", type=int, default=4096, help="rays in the CPU-baseline / PSNR sample")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--inner-iter", type=int, default=8, help="meta: inner steps (configs/train.json)")
    ap.add_argument("--support-rays", type=int, default=4000, help="meta: support rays per task")
    ap.add_argument("--query-rays", type=int, default=2000, help="meta: query rays per task")
    ap.add_argument("--data-rays", type=int, default=1 << 22, help="data: rays in the region table")
    ap.add_argument("--no-graph", action="store_true", help="c5: eager steps instead of the HIP-graph replay")
    ap.add_argument("--c5-scaling", choices=["weak", "strong"], default="weak",
                    help="c5, N > 1: every rank streams its own 1000-ray batches (weak), or the ranks split each "
                         "1000-ray batch (strong: the reference's exact runtime_adapt update)")
    ap.add_argument("--ep-capacity", choices=["adaptive", "full"], default="adaptive",
                    help="c5, N > 1: exchange segments sized per expert to ~1.5x the live pairs (overflowed steps "
                         "re-run at full capacity), or every (sender, expert) segment at the full n x S")
    ap.add_argument("--ep-graph", action="store_true",
                    help="c5, N > 1: capture the expert-parallel step, RCCL collectives included, in a HIP graph")
    ap.add_argument("--driver", choices=["step", "runtime_adapt"], default="step",
                    help="c5: time RoutedAdaptStep calls (step), or the drop-in train.runtime_adapt(steps=K) over a "
                         "loader-like list of device batches (what a reference caller of runtime_adapt gets)")
    ap.add_argument("--meta-task-order", type=int, choices=[0, 1], default=0,
                    help="meta: visit each task's support / query rays in direction-cell order (one permutation per "
                         "task and outer step; meta_train.TASK_RAY_ORDER)")
    ap.add_argument("--diag-shared-table", action="store_true",
                    help="diagnostic (c3/c4): every expert reads expert 0's hash table (one 128 MiB table instead of "
                         "K: isolates the Infinity-Cache capacity effect; outputs differ from the real render)")
    ap.add_argument("--diag-expert-box", choices=["own", "global"], default="own",
                    help="diagnostic (c3/c4): 'global' gives every expert the whole-scene box, so its hash grid has "
                         "C2's cell size instead of a ~1.9x finer one in x and y (outputs differ from the real render)")
    ap.add_argument("--diag-pixel-order", action="store_true",
                    help="diagnostic (c3): the batch in scanline pixel order instead of random order before the "
                         "expert sort")
    ap.add_argument("--diag-multi-last", action="store_true",
                    help="diagnostic (c3): the plan visits the rays whose samples reach more than one expert after "
                         "the single-expert rays (same outputs; measured slower, DESIGN.md 4k)")
    ap.add_argument("--diag-expert-only-order", action="store_true",
                    help="diagnostic (c3): sort the batch by owning expert only (no direction-cell secondary key)")
    ap.add_argument("--c5-order", choices=["none", "expert-mid"], default="none",
                    help="diagnostic (c5): visit each batch's rays sorted by (owning expert, Morton code of the ray "
                         "midpoint) -- the spatial pair order of VERDICT r03 item 7 (the loss is a mean: same update "
                         "to fp32 order)")
    ap.add_argument("--mlp-precision", choices=["fp16x3", "fp32", "amp"], default="fp16x3",
                    help="c5 / meta: training-MLP arithmetic -- fp16x3 (default, fp32-accurate), fp32 (exact), or "
                         "amp (the reference's use_amp=True: autocast(float16) products + GradScaler)")
    ap.add_argument("--dry-run", action="store_true",
                    help="launcher check: every rank reports (rank, world) over gloo and exits before any GPU call")
    a = ap.parse_args()
    if a.steps is None:
        a.steps = 200 if a.workload in ("c2", "c3") else 20
    rc = maybe_launch(sys.argv[1:], a.gpus)
    if rc is not None:
        sys.exit(rc)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != a.gpus:
        raise SystemExit(f"bench.py: --gpus {a.gpus} but the launcher started WORLD_SIZE={world} ranks")
    if a.dry_run:
        if world > 1:
            dist.init_process_group("gloo")
            t = torch.tensor([1.0])
            dist.all_reduce(t)
            world_seen = int(t.item())
            dist.destroy_process_group()
        else:
            world_seen = 1
        print(json.dumps({"dry_run": True, "rank": int(os.environ.get("RANK", "0")), "world": world,
                          "world_seen": world_seen}), flush=True)
        return
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    device = torch.device("cuda", local)
    torch.cuda.set_device(device)

    from adaptive_city_nerf_amd import ops, parallel, render_rays
    if a.mlp_precision != "fp16x3" and a.workload not in ("c5", "meta"):
        raise SystemExit("bench.py: --mlp-precision applies to the training workloads (c5, meta)")
    ops.set_train_mlp_precision(a.mlp_precision)
    S = a.samples
    K = {"c2": 1, "c3": 4, "c4": 8, "c5": 8, "c5a": 8, "occ": 1, "meta": 4, "data": 1, "clusters": 1}[a.workload]
    occ_conf = None
    if a.workload == "occ":  # nerf_runner.py:124-147 defaults: 128^3 x 4 levels, cone 0.004, step diag/1000
        occ_conf = {"use_occ": True, "resolution": 128, "levels": 4, "render_step_size": None, "cone_angle": 0.004,
                    "occ_thre": 1e-2, "alpha_thre": 1e-2, "warmup_steps": 256, "update_interval": 16}
    model, gbox, scene, sc = build_model(device, K, fill=[rank % K] if a.workload == "c5a" else None,
                                         occ_conf=occ_conf, expert_box=a.diag_expert_box)

    run_k = None   # set when the timed region is one call performing K updates (c5 --driver runtime_adapt)
    if a.diag_shared_table:
        with torch.no_grad():
            for sub in model.submodules[1:]:
                sub.xyz_encoder.hash_table.data = model.submodules[0].xyz_encoder.hash_table.data
    if a.workload == "c2":
        if a.opaque:
            with torch.no_grad():
                for sub in model.submodules:
                    sub.sigma_head.bias.add_(a.opaque)
        rays = make_rays(scene, gbox, device, a.rays, 1234 + rank)
        samples_per_step = world * a.rays * S

        def step():
            with torch.no_grad():
                return render_rays(model, rays, ray_samples=S, bg_color_default="white", early_stop_tau=a.tau)
        sample_rays = rays
    elif a.workload == "occ":
        from adaptive_city_nerf_amd import occ_ops
        sub = model.submodules[0]
        model.train()
        sub.maybe_update_occ_grid(step=0)          # warmup update: every cell's density -> binaries
        model.eval()
        sub.occ_ready = True
        rays = make_rays(scene, gbox, device, a.rays, 1234 + rank)
        with torch.no_grad():
            _, t0s, _ = sub.occupancy_marching(rays)
        occ_samples = int(t0s.numel())
        samples_per_step = world * occ_samples
        occ_frac = float(sub.occ_grid.binaries.float().mean())

        def step():
            with torch.no_grad():
                return render_rays(model, rays, bg_color_default="white", active_module=0)
        sample_rays = rays
    elif a.workload == "c3":
        # global batch (identical on every rank), sharded by owning expert; gather of rendered rays
        grays = make_rays(scene, gbox, device, world * a.rays, 1234, pixel_order=a.diag_pixel_order)
        keys = (parallel.dominant_expert(grays, model) if a.diag_expert_only_order
                else parallel.expert_spatial_keys(grays, model))
        if a.diag_multi_last:
            multi = parallel.multi_expert_rays(grays, model, S)
            keys = keys + multi.to(torch.int64) * (1 << 40)
            multi_frac = float(multi.float().mean())
        plan = parallel.expert_sorted_plan(keys, world)
        samples_per_step = grays.shape[0] * S

        def render_fn(r):
            rgb, depth, _, acc = render_rays(model, r, ray_samples=S, bg_color_default="white", _want_weights=False)
            return rgb, depth, acc

        def step():
            with torch.no_grad():
                return parallel.render_rays_sharded(grays, render_fn, plan)
        sample_rays = grays
    elif a.workload == "meta":
        # offline meta-training (configs/train.json): 4 regions x batch_size 3 tasks, 4000 support +
        # 2000 query rays, 96 samples, 8 inner steps, FOMAML, Adam param groups; expert parallel
        from types import SimpleNamespace
        from adaptive_city_nerf_amd import meta_train as MT
        from adaptive_city_nerf_amd import optim as aoptim
        S = 96 if a.samples == 256 else a.samples
        P = SimpleNamespace(algo="fomaml", ray_samples=S, chunk_points=4000000, color_space="linear",
                            optimizer="adam", lr=1e-4, encoding_lr=0.01, sigma_lr=0.002, color_lr=0.002, bg_lr=0.001,
                            weight_decay=0.0, inner_lr=0.015, inner_iter=a.inner_iter, fim=False,
                            use_amp=a.mlp_precision == "amp", grad_clip=1.0, seed=0, mixed_precision=False,
                            print_step=10 ** 9)
        # use_amp: trainer.py:24's GradScaler, replayed on the device by the graphed meta step
        meta_scaler = torch.amp.GradScaler("cuda") if P.use_amp else None
        nsup, nqry, ntask = a.support_rays, a.query_rays, 3
        pool = make_rays(scene, gbox, device, 60000, 4321)
        gen = torch.Generator(device).manual_seed(9)
        task_data = {}
        for cid in range(4):
            task_data[cid] = []
            for t in range(ntask):
                sel = torch.randint(0, pool.shape[0], (nsup + nqry,), device=device, generator=gen)
                rg = torch.rand(nsup + nqry, 3, device=device, generator=gen)
                task_data[cid].append({"support": {"rays": pool[sel[:nsup]], "rgbs": rg[:nsup]},
                                       "query": {"rays": pool[sel[nsup:]], "rgbs": rg[nsup:]}})
        model.train()
        opt = aoptim.build_optimizer(P, model)
        pg = dist.group.WORLD if world > 1 else None
        from adaptive_city_nerf_amd.expert_parallel import expert_owner
        my_regions = [c for c in range(4) if expert_owner(4, world)[c] == rank]
        samples_per_step = sum(len(task_data[c]) * (P.inner_iter * nsup + nqry) for c in range(4)) * S
        it = [0]
        # the drop-in train_step: at one process, FOMAML + FusedAdam, its first call is the eager step and
        # the later ones replay the per-region task graphs + the outer graph (meta_train.GraphedMetaStep,
        # cached on the optimizer); --no-graph: ACN_FAST_META off, every step eager
        MT.FAST_META_STEP = not a.no_graph
        MT.TASK_RAY_ORDER = a.meta_task_order

        def step():
            it[0] += 1
            import contextlib, io
            with contextlib.redirect_stdout(io.StringIO()):  # meta_update's per-region debug prints (eager)
                return MT.train_step(P, it[0], model, opt, task_data, group=pg, grad_scaler=meta_scaler)
        sample_rays = pool[:1]
        aoptim.EVENT_HOOK = []
    elif a.workload == "data":
        # TaskDataset construction over one region's device ray table (nerf_runner.py:193-201: DDA
        # routing, 1 x 5 x 5 micro-cells, image cap 0.4): HIP routing + device sort + per-cell bins
        from types import SimpleNamespace
        from adaptive_city_nerf_amd import data as adata
        # the table a DeviceRaysDataset holds: image after image, valid pixels row-major; images are the
        # validation camera at downscale 0.25 with the origin shifted per image
        H, W, intr, c2w = frame_camera(scene)
        psf = scene["pose_scale_factor"]
        n = a.data_rays
        g = torch.Generator(device).manual_seed(31 + rank)
        frames, ids, total = [], [], 0
        while total < n:
            fr, fv = ops.get_rays_image(H, W, *intr, c2w, gbox.aabb, device, near_far_override=(0.0, 100000 / psf))
            fr = fr[fv]
            fr[:, :3] += 0.05 * (torch.rand(1, 3, device=device, generator=g) - 0.5)
            ids.append(torch.full((fr.shape[0],), len(frames), dtype=torch.int32, device=device))
            frames.append(fr)
            total += fr.shape[0]
        rays = torch.cat(frames)[:n].contiguous()
        table = SimpleNamespace(_rays=rays, _rgbs=torch.rand(n, 3, device=device, generator=g),
                                _img_indices=torch.cat(ids)[:n])
        td = adata.TaskDataset(table, cell_id=rank, S_target=4000, Q_target=2000, min_rays_cell=3000,
                               image_cap=0.4, routing_policy="dda", cells=(1, 5, 5))
        samples_per_step = world * n

        def step():
            return td._route_and_bin()
        sample_rays = rays
        data_n = n
    elif a.workload == "clusters":
        # create_clusters.py per-image step at the example dataset's g22 configuration (grid 2x2, YZ
        # routing, margin 1.1, 256 samples, centred pixels, full 1536 x 2048 frames): ray generation +
        # Voronoi routing with AABB streaming; rank r routes its own images (rank-strided, no exchange
        # until the final box all-reduce)
        from adaptive_city_nerf_amd import clusters as CL
        from adaptive_city_nerf_amd.scene_box import SceneBox
        msc = scene["masks"]["g22_grid_bm110_ss11"]
        cl_cents = torch.tensor(msc["centroids"], dtype=torch.float32)
        cl_box = SceneBox(aabb=torch.tensor(msc["aabb_global"], dtype=torch.float32).to(device))
        cam = scene["val_cam0"]
        cl_md = {"H": cam["H"], "W": cam["W"], "intrinsics": torch.tensor(cam["intrinsics"], dtype=torch.float32),
                 "c2w": torch.tensor(cam["c2w"], dtype=torch.float32)}
        S = 256
        Cn = cl_cents.shape[0]
        cl_state = [torch.full((Cn, 3), float("inf"), device=device), torch.full((Cn, 3), float("-inf"), device=device),
                    torch.zeros(Cn, dtype=torch.int64, device=device), torch.zeros(Cn, dtype=torch.int32, device=device)]
        data_n = cam["H"] * cam["W"]
        samples_per_step = world * data_n * S

        def step():
            rays, valid = CL.image_rays(cl_md, True, cl_box, (None, None), device)
            bits = CL.voronoi_route(rays, S, cl_cents, True, 1.1, update_aabbs=True, mins_out=cl_state[0],
                                    maxs_out=cl_state[1], counts_out=cl_state[2], nan_out=cl_state[3])
            return bits, valid, rays
        sample_rays = None
    elif a.workload == "c5":
        # BASELINE C5 as runtime_adapt runs it (runtime_adapt.py:286-309): the routed 8-expert container
        # (no active_module) adapted on 1000-ray batches x 96 samples streamed from a continual batch of
        # many cameras; targets = the render of a different ("changed city") 8-expert model, so the
        # val PSNR after the timed steps measures real adaptation
        from types import SimpleNamespace
        from adaptive_city_nerf_amd import optim as aoptim
        from adaptive_city_nerf_amd.train import adapt_step
        S = 96 if a.samples == 256 else a.samples      # configs/eval.json:15 ray_samples
        P = SimpleNamespace(ray_samples=S, chunk_points=4000000, color_space="linear", optimizer="adam", lr=1e-4,
                            encoding_lr=0.01, sigma_lr=0.002, color_lr=0.002, bg_lr=0.001, weight_decay=0.0)
        nb, bsz = 32, 1000
        strong = a.c5_scaling == "strong" and world > 1
        # weak: every rank streams its own 1000-ray batches (global batch W x 1000); strong: the ranks split
        # each 1000-ray runtime_adapt batch (the reference's exact update), so they share one pool
        pool = make_rays_multi(gbox, device, nb * bsz, 4321 + (0 if strong else rank)).view(nb, bsz, 8)
        val_rays = make_rays_multi(gbox, device, 4096, 97)
        teacher, _, _, _ = build_model(device, K, seed=1, table_seed=900)
        with torch.no_grad():
            gtp = render_rays(teacher, pool.view(-1, 8), ray_samples=S, _want_weights=False)[0].view(nb, bsz, 3)
            gt_val = render_rays(teacher, val_rays, ray_samples=S, _want_weights=False)[0]
        del teacher
        torch.cuda.empty_cache()

        def val_psnr():
            from adaptive_city_nerf_amd.color_space import color_space_transformer
            model.eval()
            with torch.no_grad():
                pr = render_rays(model, val_rays, ray_samples=S, _want_weights=False)[0]
            model.train()
            p_, g_ = color_space_transformer(pr, gt_val, color_space="linear")
            return float(-10.0 * torch.log10(torch.mean((p_.double() - g_.double()) ** 2).clamp_min(1e-8)))
        psnr_before = val_psnr()
        model.train()
        opt = aoptim.build_optimizer(P, model)
        samples_per_step = (1 if strong else world) * bsz * S
        it = [0]
        graphed = None
        expert = None
        routed = None
        ep = None
        pg = dist.group.WORLD if world > 1 else None
        shard = slice(bsz * rank // world, bsz * (rank + 1) // world) if strong else slice(0, bsz)
        if world > 1:   # one expert block per GPU, fixed-capacity exchanges, no host synchronisation
            from adaptive_city_nerf_amd.expert_parallel import ExpertParallelAdaptStep
            ep = ExpertParallelAdaptStep(P, model, shard.stop - shard.start, opt,
                                         n_rays_global=bsz if strong else world * bsz, grad_clip=1.0, group=pg,
                                         graph=a.ep_graph, warmup=2,
                                         capacity=None if a.ep_capacity == "full" else "adaptive")
        if a.c5_order == "expert-mid":
            def morton_mid(r):
                near, far = r[:, 6], r[:, 7]
                mid = r[:, :3] + r[:, 3:6] * torch.where(torch.isfinite(far), 0.5 * (near + far),
                                                         torch.zeros_like(near)).unsqueeze(1)
                lo, hi = mid.min(0).values, mid.max(0).values
                q = ((mid - lo) / (hi - lo).clamp_min(1e-12) * 1023).clamp(0, 1023).long()
                code = torch.zeros(r.shape[0], dtype=torch.int64, device=r.device)
                for b in range(10):
                    for ax in range(3):
                        code |= ((q[:, ax] >> b) & 1) << (3 * b + ax)
                return parallel.dominant_expert(r, model).to(torch.int64) * (1 << 30) + code
            with torch.no_grad():
                for i in range(nb):
                    o = torch.argsort(morton_mid(pool[i]))
                    pool[i] = pool[i][o]
                    gtp[i] = gtp[i][o]
        loader = [(pool[i], gtp[i]) for i in range(nb)]   # a runtime_adapt data loader's batches (device)
        if world == 1 and a.driver == "step":  # the whole routed step (no host sync), one HIP graph (eager: --no-graph)
            from adaptive_city_nerf_amd.routed_train import RoutedAdaptStep
            routed = RoutedAdaptStep(P, model, bsz, opt, grad_clip=1.0, graph=not a.no_graph, warmup=2)
        if a.driver == "runtime_adapt":
            if world > 1:
                raise SystemExit("bench.py: --driver runtime_adapt is the single-process drop-in (the reference's "
                                 "runtime_adapt has no process group); use --driver step for N > 1")
            from adaptive_city_nerf_amd import train as atrain

            def run_k(k):    # ONE drop-in call performing k updates, cycling over the loader
                return atrain.runtime_adapt(P=P, model=model, data_loader=loader, optimizer=opt, steps=k)

        def step():
            # N > 1: the experts distributed over the ranks (expert_parallel.py), every rank streaming
            # its own 1000-ray batches of the global batch
            i = it[0] % nb
            it[0] += 1
            if routed is not None:
                return routed(pool[i], gtp[i])
            if ep is not None:
                return ep(pool[i][shard], gtp[i][shard])
            return adapt_step(P, model, pool[i], gtp[i], opt, grad_clip=1.0, group=pg)
        sample_rays = pool[0]
        aoptim.EVENT_HOOK = []
    elif a.workload == "c5a":
        from types import SimpleNamespace
        from adaptive_city_nerf_amd import optim as aoptim
        from adaptive_city_nerf_amd.train import adapt_step
        S = 96 if a.samples == 256 else a.samples      # configs/eval.json:15 ray_samples
        P = SimpleNamespace(ray_samples=S, chunk_points=4000000, color_space="linear", optimizer="adam", lr=1e-4,
                            encoding_lr=0.01, sigma_lr=0.002, color_lr=0.002, bg_lr=0.001, weight_decay=0.0)
        nb, bsz = 32, 1000
        pool = make_rays(scene, gbox, device, nb * bsz, 4321 + rank).view(nb, bsz, 8)
        gtp = torch.rand(nb, bsz, 3, device=device, generator=torch.Generator(device).manual_seed(5 + rank))
        model.train()
        opt = aoptim.build_optimizer(P, model)
        shared = list(model.bg_mlp.parameters())
        pg = dist.group.WORLD if world > 1 else None
        expert = rank % K
        samples_per_step = world * bsz * S
        it = [0]

        graphed = None
        if not a.no_graph:  # the launch-bound step replayed as one HIP graph (no collective in this variant)
            from adaptive_city_nerf_amd.train import GraphedAdaptStep
            graphed = GraphedAdaptStep(P, model, pool[0], gtp[0], opt, active_module=expert, grad_clip=1.0,
                                       warmup=2)

        def step():
            i = it[0] % nb
            it[0] += 1
            if graphed is not None:
                return graphed(pool[i], gtp[i])
            return adapt_step(P, model, pool[i], gtp[i], opt, active_module=expert, grad_clip=1.0)
        sample_rays = pool[0]
        aoptim.EVENT_HOOK = []
    else:
        H, W, intr, c2w = frame_camera(scene, a.frame, a.frame)
        samples_per_step = H * W * S
        ep_stats = {}   # --layout expert: the planned exchange's bytes of the last frame
        gt = torch.rand(H, W, 3, device=device, generator=torch.Generator(device).manual_seed(7))

        def step():
            with torch.no_grad():
                if a.layout == "expert":
                    from adaptive_city_nerf_amd.expert_parallel import render_image_expert_parallel
                    return render_image_expert_parallel(model, H=H, W=W, fx=intr[0], fy=intr[1], cx=intr[2],
                                                        cy=intr[3], c2w=c2w, scene_box=gbox, ray_samples=S,
                                                        gt_srgb=gt, group=dist.group.WORLD if world > 1 else None,
                                                        stats=ep_stats)
                return parallel.render_image_sharded(model, H=H, W=W, fx=intr[0], fy=intr[1], cx=intr[2], cy=intr[3],
                                                     c2w=c2w, scene_box=gbox, ray_samples=S, gt_srgb=gt)
        frays, fvalid = ops.get_rays_image(H, W, *intr, c2w, gbox.aabb, device, near_far_override=(None, None))
        sample_rays = frays

    if run_k is not None:
        out = run_k(a.warmup)
    else:
        for _ in range(a.warmup):
            out = step()
    torch.cuda.synchronize()
    # c2: one acn call per step, timed by two HIP events bracketing the K timed calls on the launch stream
    # (a per-call event pair costs ~8 us of queue time per step, 2.5% of a C2 step: tools/event_overhead.py)
    bracket = a.workload == "c2"
    ops.EVENT_HOOK = None if bracket else []
    if a.workload == "occ":
        occ_ops.EVENT_HOOK = ops.EVENT_HOOK
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    mark = os.environ.get("ACN_TRACE_MARK") == "1"   # tools/trace_busy.py: bracket the timed steps in a kernel trace
    if mark:
        torch.cuda._sleep(1000)
    t0 = time.perf_counter()
    if bracket:
        eb = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        eb[0].record()
    if run_k is not None:
        out = run_k(a.steps)
    else:
        for _ in range(a.steps):
            out = step()
    if bracket:
        eb[1].record()
    if mark:
        torch.cuda._sleep(1000)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    if a.workload == "c5a" and graphed is not None:
        # graph replays run no Python, so the Adam launch is timed by one eager step afterwards
        from adaptive_city_nerf_amd import optim as aoptim
        graphed.sync_state()
        opt._graph = None
        aoptim.EVENT_HOOK = []
        adapt_step(P, model, pool[0], gtp[0], opt, active_module=expert, grad_clip=1.0)
        torch.cuda.synchronize()
    if a.workload == "c5" and run_k is not None:   # the step object the drop-in call built and replayed
        routed = next(iter(opt._acn_routed_steps.values()), None)
    if a.workload == "c5" and routed is not None:
        # graph replays run no Python: the Adam launch is timed by eager steps of the same object
        from adaptive_city_nerf_amd import routed_train as RT
        graph_was = routed.graph
        routed.graph = None
        RT.EVENT_HOOK = aoptim.EVENT_HOOK = []
        RT.BWD_HOOK = []
        for _ in range(3):
            step()
        torch.cuda.synchronize()
        hash_bwd_ms = float(np.mean([e0.elapsed_time(e1) for e0, e1 in RT.BWD_HOOK]))
        hash_segments = hash_bwd_segments(routed)
        RT.EVENT_HOOK = RT.BWD_HOOK = None
    if a.workload == "c5" and ep is not None:
        # the Adam launch of the expert-parallel step, timed by eager steps (collective: every rank runs them)
        from adaptive_city_nerf_amd import routed_train as RT
        ep.graph = None
        RT.EVENT_HOOK = aoptim.EVENT_HOOK = []
        for _ in range(3):
            step()
        torch.cuda.synchronize()
        RT.EVENT_HOOK = None
    if a.workload == "meta":
        # graph replays run no Python: the fused MLP backward (the step's dominant kernel) and the outer Adam
        # launch are timed by eager steps afterwards
        import contextlib, io
        graphed_meta = opt.__dict__.get("_acn_meta_graph") or None
        if graphed_meta is not None:
            graphed_meta.sync_state()
        MT.FAST_META_STEP = False
        aoptim.EVENT_HOOK = []
        ops.DW_HOOK = []
        with contextlib.redirect_stdout(io.StringIO()):
            for _ in range(3):
                it[0] += 1
                MT.train_step(P, it[0], model, opt, task_data, group=pg, grad_scaler=meta_scaler)
        torch.cuda.synchronize()
        dw_hook, ops.DW_HOOK = ops.DW_HOOK, None
        dw_ms = float(np.mean([e0.elapsed_time(e1) for e0, e1, _, _ in dw_hook]))
        dw_flop = float(np.mean([ops.mlp_bwd_flops(m, wh) for _, _, m, wh in dw_hook]))
        dw_samples = float(np.mean([m for _, _, m, _ in dw_hook]))
        dw_launches = len(dw_hook) // 3
    if a.workload == "c5":
        psnr_after = val_psnr()
    if a.workload in ("c5", "c5a", "meta"):
        from adaptive_city_nerf_amd import optim as aoptim
        hook = aoptim.EVENT_HOOK[-a.steps:]
        aoptim.EVENT_HOOK = None
    elif bracket:
        hook = [(eb[0], eb[1])] * a.steps     # one launch per step; average = bracketed time / K
    else:
        hook = ops.EVENT_HOOK
    # an entry is one or more (start, end) event pairs of one step's launches (the split Adam: early + late pass)
    kernel_ms = float(np.mean([sum(ev[i].elapsed_time(ev[i + 1]) for i in range(0, len(ev), 2)) for ev in hook]))
    if bracket:
        kernel_ms /= a.steps
    if a.workload == "data":
        # route_kernel (~0.1 ms) is shorter than the host gap between a per-call event and its launch
        # (the step syncs for the bin counts, so the queue is empty): time it back to back instead
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        ev[0].record()
        for _ in range(a.steps):
            adata.route_rays(rays, td.aabb, td.cells, td.assignment_checkpoint, td.routing_policy)
        ev[1].record()
        torch.cuda.synchronize()
        kernel_ms_gapped, kernel_ms = kernel_ms, ev[0].elapsed_time(ev[1]) / a.steps
    kernel_launches = len(hook) // max(a.steps, 1)
    ops.EVENT_HOOK = None
    if world > 1:
        t = torch.tensor([dt, kernel_ms], device=device, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt, kernel_ms = float(t[0]), float(t[1])

    value = samples_per_step * a.steps / dt
    ms_per_step = dt / a.steps * 1e3
    if a.workload == "c5":      # Adam updates every parameter that received a gradient (the hit experts + head)
        if routed is not None:
            counts = routed.seg[K + 1: 2 * K + 1].cpu().tolist()
            experts_hit = sum(1 for c in counts if c > 0)
            nparam = sum(r[0].numel() for r, f in zip(routed.rows, routed.flags.cpu().tolist())
                         if (f & 0xffff) >= K or counts[f & 0xffff] > 0)
        elif ep is not None:   # this rank's Adam: its owned experts that received pairs + the head
            counts = ep.eseg[ep.E + 1: 2 * ep.E + 1].cpu().tolist()
            experts_hit = sum(1 for c in counts if c > 0)
            nparam = sum(r[0].numel() for r, f in zip(ep.adam.rows, ep.adam.flags.cpu().tolist())
                         if (f & 0xffff) >= ep.E or counts[f & 0xffff] > 0)
        else:
            nparam = sum(p.numel() for p in model.parameters() if p.grad is not None)
            experts_hit = sum(1 for sub in model.submodules if sub.xyz_encoder.hash_table.grad is not None)
        adam_bytes = 28 * nparam            # read p, g, m, v + write p, m, v (fp32)
        adam_bytes_dense = adam_bytes
        segmap = None
        if routed is not None and getattr(routed, "segmaps", None) is not None:
            # segment-mapped Adam (optim.hip adam_chunk_seg): a 64-B table segment never touched is skipped;
            # one touched before but not this step reads + writes p, m, v (384 B); one touched this step also
            # reads g and clears it (+128 B); both byte maps are read for every segment of a hit table
            ever, total = routed.segment_stats()
            ntab = sum(sub.xyz_encoder.hash_table.numel() for k_, sub in enumerate(model.submodules)
                       if counts[k_] > 0)
            nseg = ntab // 16
            now = hash_segments
            adam_bytes = 28 * (nparam - ntab) + 384 * ever + 128 * now + 2 * nseg
            ever_lines = routed.segment_line_stats()
            segmap = {"table_segments_hit_experts": nseg, "ever_touched_segments": ever,
                      "ever_touched_128B_lines": ever_lines,
                      "ever_touched_fraction": round(ever / max(total, 1), 4),
                      "segments_touched_this_step": now, "adam_bytes_dense": adam_bytes_dense,
                      "adam_bytes_segmap": adam_bytes,
                      "note": "ever-touched counted after the timed steps (it only grows); this-step segments = "
                              "the distinct 64-B segments of one step's table scatter (hash_bwd_segments)"}
        achieved_gbs = adam_bytes / (kernel_ms * 1e-3) / 1e9
    if a.workload == "c5a":
        nparam = sum(p.numel() for p in model.submodules[expert].parameters()) + sum(p.numel() for p in shared)
        adam_bytes = 28 * nparam            # read p, g, m, v + write p, m, v (fp32)
        achieved_gbs = adam_bytes / (kernel_ms * 1e-3) / 1e9
    if a.workload == "clusters":  # fp32 VALU arithmetic per sample: t, x, |x|^2 (10) + per centroid dot + d2 (7)
        cl_flop = 10 + Cn * 7
        cl_achieved = cl_flop * data_n * S / (kernel_ms * 1e-3) / 1e12
    if a.workload == "data":  # route_kernel: read a ray (32 B), write cell id (8 B) + flags (1 B)
        route_bytes = 41 * data_n
        achieved_gbs = route_bytes / (kernel_ms * 1e-3) / 1e9
    if a.workload == "meta":  # the outer Adam updates the experts of this rank's regions + the shared head
        nparam = sum(p.numel() for c in my_regions for p in model.submodules[c].parameters()) + \
            sum(p.numel() for p in model.bg_mlp.parameters())
        adam_bytes = 28 * nparam
        achieved_gbs = adam_bytes / (kernel_ms * 1e-3) / 1e9
    # samples one launch of the dominant kernel processes on this rank
    launch_samples = samples_per_step // world // max(kernel_launches, 1)
    achieved = FLOP_PER_SAMPLE * launch_samples / (kernel_ms * 1e-3) / 1e12
    tr = render_traffic_profile(a.workload, S, a.layout) if a.workload in ("c2", "c3", "c4") else None
    kname = {"c5": "adam_slots_kernel (Adam over every expert with routed samples + background head, clip coefficient "
                   "folded in, table gradients cleared in the same pass)",
             "c5a": "adam_kernel (fused clip + Adam over the adapted expert + background head)",
             "c2": "ray_order_kernel + render_ws_kernel<1> (one acn_render_stratified_fwd_ordered call: direction "
                   "grouping of the batch, then the fused stratified render, 1 expert, the workgroup's 16 rays "
                   "sharing their field tiles, each tile 8 rays x 4 consecutive samples; kernel_ms = two HIP events "
                   "bracketing the K timed calls on the launch stream / K)",
             "c3": "render_wss_kernel (fused stratified render, soft routing over 4 experts, two staged per round, "
                   "field tiles of 8 rays x 4 consecutive samples)",
             "c4": ("ep_field_kernel (the owned expert's fused MFMA field over the received per-sample records; "
                    "one-expert-per-GPU layout, kernel_ms per launch)"
                    if a.layout == "expert" else
                    "render_wss_kernel (fused stratified render, soft routing over 8 experts, two staged per round, "
                    "field tiles of 8 rays x 4 consecutive samples)"),
             "occ": "occ_render_kernel<1,1,0> (fused occupancy render over packed marched samples, 1 expert)",
             "meta": "adam_kernel (fused clip + Adam of the outer meta-update over the region experts + shared head)",
             "data": "route_kernel (TaskDataset region clip + DDA max-overlap micro-cell routing + keep tolerance)",
             "clusters": "voronoi_kernel<4,2> (create_clusters Voronoi routing, 256 samples x 4 centroids per ray, "
                         "AABB streaming)"
             }[a.workload]
    # The fused render is bound by gathering hash-table lines from beyond the XCD L2 (Infinity Cache,
    # the tables are cache-resident): PMC shows TD busy and stalled on the texture cache while the MFMA
    # pipe is mostly idle (profiles/pmc_render_r02.json).  `achieved` is the ALGORITHMIC table bytes
    # (1024 B/sample) against HBM peak; the measured line traffic against the
    # Infinity-Cache row-gather rate and the fp32-MFMA fraction ride along.
    hash_gbs = BYTES_PER_SAMPLE * launch_samples / (kernel_ms * 1e-3) / 1e9
    roofline = {"bound": "hbm", "achieved": round(hash_gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(hash_gbs / HBM_PEAK_GBS, 4),
                "traffic": (tr or {}).get("hbm_bytes_per_launch")
                if tr and tr.get("samples_per_launch") == int(launch_samples) else None,
                "kernel": kname, "kernel_ms": round(kernel_ms, 4), "samples_per_launch": int(launch_samples),
                "bytes_per_sample": BYTES_PER_SAMPLE,
                "bytes_algorithmic_per_launch": int(BYTES_PER_SAMPLE * launch_samples),
                "secondary": {"bound": "mfma", "unit": "TFLOP/s", "achieved": round(achieved, 2),
                              "peak": FP32_MFMA_PEAK_TFLOPS, "frac": round(achieved / FP32_MFMA_PEAK_TFLOPS, 4),
                              "flop_per_sample": FLOP_PER_SAMPLE,
                              "mlp_arith": "fp32-accurate 3-term fp16 split (hi*hi + hi*lo + lo*hi) on "
                                           "v_mfma_f32_32x32x16_f16, fp32 accumulate (DESIGN.md 4)"}}
    gc = load_gather_ceiling() if a.workload == "c2" else None
    if gc:
        # calibrated ceiling of THIS access shape: the render's hash gathers alone, same sample
        # points, table and lane mapping (tools/micro/hash_gather.hip), best of a sweep over levels in flight x
        # waves per CU x XCD bands; same algorithmic bytes, so frac = ceiling time / render time
        c = gc["ceiling"]
        roofline["gather_ceiling"] = {
            "what": "gather-only kernel issuing the fused render's exact hash-table access (8-B corner rows, 16 "
                    "levels x 8 corners, 128 MiB fp32 table, 32-sample tiles, half-wave per 8 levels, XCD bands) "
                    "over the C2 sample points, no MLP / compositing; best of levels-in-flight 1-4 x 4-16 waves/CU "
                    "x bands on/off",
            "ceiling_ms": c["config"]["ms"], "ceiling_alg_gbs": c["alg_gbs"], "best_config": c["config"],
            "achieved_alg_gbs": round(hash_gbs, 1), "frac": round(hash_gbs / c["alg_gbs"], 4),
            "uniform_random_points_alg_gbs": gc["uniform_best"]["alg_gbs"],
            "source": "profiles/r03_hash_gather_ceiling.json (+ r03_rocprof_hash_gather_kernel_stats.csv)"}
    if tr and tr.get("samples_per_launch") == int(launch_samples):
        d = tr.get("derived", {})
        miss_bytes = d.get("l2_miss_bytes_per_launch_at_128B")
        prof_ms = (tr.get("rocprof_avg_ns") or 0.0) / 1e6
        roofline["traffic_detail"] = {
            "what": "bytes beyond the XCD L2s per launch: 2 x FETCH_SIZE (gfx950 read correction, "
                    "MI355X_MICROARCH.md 'HBM') + WRITE_SIZE, Infinity-Cache hits included; cross-checked by "
                    "TCC_MISS x 128 B",
            "source": f"{tr['_source']} ({tr.get('round')}, kernel {tr.get('kernel_match')})",
            "traffic_over_algorithmic": round(d.get("traffic_over_algorithmic", 0.0), 3),
            "fetch_over_tcc_miss_lines": round(d.get("fetch_corrected_over_tcc_miss_lines") or 0.0, 3),
            "l2_misses_per_sample": round(d.get("l2_misses_per_sample", 0.0), 2),
            "l2_requests_per_sample": round(d.get("l2_requests_per_sample", 0.0), 2),
            "l2_hit_rate": round(d.get("l2_hit_rate") or 0.0, 3),
            "td_busy_frac": round(d.get("td_busy_frac") or 0.0, 3),
            "td_stalled_on_tc_frac": round(d.get("td_stalled_on_tc_frac") or 0.0, 3),
            "mfma_busy_frac_per_simd": round(d.get("mfma_busy_frac_per_simd") or 0.0, 3),
            "mean_waves_per_cu": round(d.get("mean_waves_per_cu") or 0.0, 2),
            "profiled_kernel_ms": round(prof_ms, 4),
            "traffic_gbs_at_profiled_time": round(tr["hbm_bytes_per_launch"] / (prof_ms * 1e-3) / 1e9, 1)
            if prof_ms else None,
            "line_bytes_per_launch": int(miss_bytes) if miss_bytes else None}
    if a.workload in ("c5", "c5a", "meta"):
        roofline = {"bound": "hbm", "achieved": round(achieved_gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": round(achieved_gbs / HBM_PEAK_GBS, 4), "traffic": None, "kernel": kname,
                    "kernel_ms": round(kernel_ms, 4), "params_per_launch": int(nparam),
                    "bytes_per_param": 28, "bytes_algorithmic_per_launch": int(adam_bytes)}
        if a.workload == "c5":
            pmc = load_traffic("c5", "r02") or {}
            ad = pmc.get("adam_slots_kernel", {})
            if ad.get("params") == int(nparam) and segmap is None:   # counters of this exact workload (dense Adam)
                roofline["traffic"] = ad["hbm_bytes_per_launch"]
            if segmap is not None:
                roofline["bytes_per_param"] = "28 dense (MLP, head); table segments per segmap"
                roofline["segmap"] = segmap
                try:   # round-4 counters of the segment-mapped pass on this workload (tools/gpu_r04ai.sh)
                    ad4 = json.loads((REPO / "profiles" / "r04_pmc_c5_adam.json").read_text())
                except Exception:
                    ad4 = None
                if ad4 is not None and routed is not None and world == 1:
                    roofline["traffic"] = ad4["traffic_bytes"]
                    roofline["traffic_detail"] = {
                        "source": "profiles/r04_pmc_c5_adam.json", "read_bytes": ad4["read_bytes"],
                        "write_bytes": ad4["write_bytes"], "traffic_over_algorithmic_at_profile":
                            ad4["traffic_over_algorithmic"], "correction": ad4["correction"]}
                    pmc = dict(pmc)
                    pmc["hashgrid_bwd_pairs"] = {"atomic_requests_per_launch":
                                                 ad4["hashgrid_bwd_pairs"]["atomic_requests_per_launch"],
                                                 "_src": "profiles/r04_pmc_c5_adam.json (TCC_EA0_ATOMIC_sum)"}
            hb = pmc.get("hashgrid_bwd_pairs", {})
            roofline["secondary"] = {
                "kernel": "hashgrid_bwd_pairs (table-gradient scatter-add, returning float atomics that also telescope the tables share of the clip norm)",
                "bound": "memory-side atomic request rate: 1.3 TB/s of added bytes = 4 x 64-B requests per 256-B "
                         "wave-instruction = ~20.3 G requests/s chip-wide (MI355X_MICROARCH.md 'Global float "
                         "atomics'; 64 rows per instruction at 0.08 TB/s is the same request rate)",
                "peak_requests_per_s": ATOMIC_REQ_PEAK,
                "atomic_requests_per_launch": hb.get("atomic_requests_per_launch"),
                "requests_source": pmc.get("hashgrid_bwd_pairs", {}).get("_src",
                                           "profiles/pmc_c5_r02.json (TCC_EA0_ATOMIC_sum, same workload)")}
            if routed is not None:
                sec = roofline["secondary"]
                sec["kernel_ms"] = round(hash_bwd_ms, 4)
                sec["distinct_segments_per_launch"] = hash_segments
                sec["floor_ms_at_peak"] = round(hash_segments / ATOMIC_REQ_PEAK * 1e3, 4)
                sec["frac_vs_segment_floor"] = round(hash_segments / ATOMIC_REQ_PEAK * 1e3 / hash_bwd_ms, 4)
                if sec["atomic_requests_per_launch"]:
                    sec["requests_over_distinct_segments"] = round(sec["atomic_requests_per_launch"] / hash_segments, 3)
                    sec["achieved_requests_per_s"] = round(sec["atomic_requests_per_launch"] / (hash_bwd_ms * 1e-3), 1)
    if a.workload == "meta":
        # dominant kernel: the fused MLP backward (mlp_bwd_dw_pc_kernel, ~40% of the step); FLOP roofline on the
        # algorithmic dW + dX MACs x 2 (ops.mlp_bwd_flops) against the fp32 matrix peak (the products are
        # fp32-accurate: fp16x3 split for dX, fp32 MFMA for dW); the forward recompute is stated beside it
        dw_tf = dw_flop / (dw_ms * 1e-3) / 1e12
        adam = roofline
        roofline = {"bound": "mfma", "achieved": round(dw_tf, 2), "peak": FP32_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s",
                    "frac": round(dw_tf / FP32_MFMA_PEAK_TFLOPS, 4), "traffic": None,
                    "kernel": "mlp_bwd_dw_pc_kernel (fused MLP backward, producer / consumer waves: forward recompute "
                              "+ dX chain on the fp16x3 split in waves 0-3, dW + db on fp32 MFMA in waves 4-7; "
                              "kernel_ms = HIP events around the acn_mlp_train_bwd_dw call = weight pack + "
                              "mlp_bwd_dw_pc_kernel + mlp_dw_reduce_kernel)",
                    "kernel_ms": round(dw_ms, 4), "launches_per_step": dw_launches,
                    "share_of_step": round(dw_ms * dw_launches / ms_per_step, 4),
                    "samples_per_launch": int(dw_samples), "flop_per_launch": int(dw_flop),
                    "flop_per_sample": {"dW": 2 * ops.MLP_BWD_MACS_DW, "dX": 2 * ops.MLP_BWD_MACS_DX,
                                        "dX_h0_when_wanted": 2 * ops.MLP_BWD_MACS_DX0},
                    "recompute_flop_per_sample_not_counted": 2 * ops.MLP_FWD_MACS,
                    "achieved_incl_recompute": round((dw_flop + 2 * ops.MLP_FWD_MACS * dw_samples)
                                                     / (dw_ms * 1e-3) / 1e12, 2),
                    "secondary": adam}
    if a.workload == "clusters":
        roofline = {"bound": "mfma", "achieved": round(cl_achieved, 2), "peak": FP32_MFMA_PEAK_TFLOPS,
                    "unit": "TFLOP/s", "frac": round(cl_achieved / FP32_MFMA_PEAK_TFLOPS, 4),
                    "traffic": (load_traffic("clusters") or {}).get("hbm_bytes_per_launch"),
                    "kernel": kname, "kernel_ms": round(kernel_ms, 4), "rays_per_launch": int(data_n),
                    "flop_per_sample": cl_flop, "note": "fp32 VALU (no matrix shape: K = 2); MI355X's FP32 vector "
                                                        "peak equals its FP32 matrix peak"}
    if a.workload == "data":
        roofline = {"bound": "hbm", "achieved": round(achieved_gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": round(achieved_gbs / HBM_PEAK_GBS, 4),
                    "traffic": (load_traffic("data") or {}).get("hbm_bytes_per_launch"), "kernel": kname,
                    "kernel_ms": round(kernel_ms, 4), "kernel_ms_in_step_events": round(kernel_ms_gapped, 4),
                    "rays_per_launch": int(data_n), "bytes_per_ray": 41,
                    "bytes_algorithmic_per_launch": int(route_bytes)}

    cpu, psnr, rmse, maxerr = None, None, None, None
    if rank == 0 and not a.no_cpu_baseline and a.workload in ("c5", "c5a"):
        cpu = cpu_baseline_train(model, sc, pool[0], gtp[0], S, expert, a.cpu_seconds)
    if rank == 0 and not a.no_cpu_baseline and a.workload == "occ":
        idx = torch.arange(rays.shape[0], device=device)[: a.cpu_rays]
        cpu, psnr, rmse, maxerr = cpu_baseline_occ(model, rays[idx], out[0][idx].cpu().numpy(), a.cpu_seconds)
    if rank == 0 and not a.no_cpu_baseline and a.workload == "meta":
        cpu = cpu_baseline_meta(model, sc, task_data, S, a.cpu_seconds)
    if rank == 0 and not a.no_cpu_baseline and a.workload == "clusters":
        cpu = cpu_baseline_clusters(out, cl_cents, S, a.cpu_seconds)
    if rank == 0 and not a.no_cpu_baseline and a.workload == "data":
        cpu = cpu_baseline_data(td, rays, out, a.cpu_seconds)
    if rank == 0 and not a.no_cpu_baseline and a.workload not in ("c5", "c5a", "occ", "meta", "data", "clusters"):
        rgb_all = out[0].reshape(-1, 3)
        if a.workload == "c2":
            idx = torch.arange(rays.shape[0], device=device)[: a.cpu_rays]
        else:  # a bounded random sample of the gathered frame / batch (valid rays)
            fin = torch.nonzero(torch.isfinite(sample_rays[:, 7])).squeeze(1).cpu()
            g = torch.Generator().manual_seed(99)
            idx = fin[torch.randperm(fin.numel(), generator=g)[: a.cpu_rays]].to(device)
        cpu, psnr, rmse, maxerr = cpu_baseline(model, sc, sample_rays[idx], S, rgb_all[idx].cpu().numpy(),
                                               a.cpu_seconds)

    if rank == 0:
        cfg = {"c2": {"workload": "C2: single Instant-NGP expert, 4096 rays x 256 samples per GPU, eval, fused "
                                  "render_rays" + (f", early ray termination tau={a.tau}" if a.tau > 0 else "")
                                  + (f", opaque variant (sigma_head bias +{a.opaque})" if a.opaque else ""),
                      "rays_per_gpu": a.rays, "experts": 1},
               "c3": {"workload": "C3: 2x2 Voronoi grid -> 4 experts (soft routing bm 1.05), 4096 rays x 256 samples "
                                  "per GPU sharded by owning expert, RCCL all-gather of rendered rays",
                      "rays_per_gpu": a.rays, "experts": 4},
               "c4": {"workload": f"C4: 4x2 grid -> 8 experts (synthetic layout), {a.frame}x{a.frame} frame x "
                                  f"{S} samples, " + ("experts distributed one per GPU: all-to-all of per-sample "
                                                      "records + RCCL all-gather + PSNR all-reduce"
                                                      if a.layout == "expert" else
                                                      "experts replicated, rays sharded by owning expert, RCCL "
                                                      "all-gather + PSNR all-reduce"), "layout": a.layout,
                      "frame": [a.frame, a.frame], "experts": 8},
               "c5": {"workload": f"C5: online adaptation (runtime_adapt), the routed 8-expert container (soft routing, "
                                  f"no active_module) on 1000-ray x {S}-sample batches from a 249-camera stream: "
                                  f"train render + MSE + backward + fused clip/Adam over every expert hit"
                                  + ("; timed as ONE drop-in train.runtime_adapt(steps=K) call over a loader-like "
                                     "list of device batches" if a.driver == "runtime_adapt" else ""),
                      "rays_per_step_per_gpu": 1000 // world if (a.c5_scaling == "strong" and world > 1) else 1000,
                      "experts": 8, "driver": a.driver,
                      "layout": ("one expert block per GPU: fixed-capacity all-to-alls of pair records, no host "
                                 "synchronisation (expert_parallel.ExpertParallelAdaptStep)"
                                 + (", captured with its RCCL collectives" if a.ep_graph else "")) if world > 1
                      else "single GPU: routed_train.RoutedAdaptStep"
                      + ("" if a.no_graph else " replayed as one HIP graph"),
                      "scaling_mode": a.c5_scaling if world > 1 else None},
               "c5a": {"workload": f"C5a (placement variant, not a reference configuration): rank r adapts expert r "
                                  f"alone (active_module) on its own 1000-ray x {S}-sample batches, no collective "
                                  f"(train render + MSE + backward + fused clip/Adam); the step replayed as one HIP graph"
                                  f"{' (disabled)' if a.no_graph else ''}", "rays_per_step_per_gpu": 1000,
                      "experts": 8},
               "occ": {"workload": f"occupancy renderer (render_expert_occ): {a.rays} rays per GPU marched through a "
                                   f"128^3 x 4-level grid (warmup-updated from the field, "
                                   f"{100 * occ_frac if a.workload == 'occ' else 0:.1f}% cells occupied), step "
                                   f"diag/1000, cone 0.004; metric counts marched samples",
                       "rays_per_gpu": a.rays, "experts": 1,
                       "marched_samples_per_gpu": occ_samples if a.workload == "occ" else None},
               "meta": {"workload": "offline meta-training step (meta_train_step.train_step, configs/train.json): 4 "
                                    "regions x 3 tasks, 4000 support + 2000 query rays x 96 samples, 8 inner FOMAML "
                                    "steps, outer clip + Adam; metric = trained ray-samples (fwd+bwd) per second; 1 "
                                    "GPU: per-region task graphs + outer graph (meta_train.GraphedMetaStep)"
                                    + (" (disabled)" if a.no_graph else ""),
                        "experts": 4, "regions": 4, "tasks_per_region": 3,
                        "inner_iter": a.inner_iter if a.workload == "meta" else None,
                        "task_ray_order": "direction cells" if a.meta_task_order else "as drawn"},
               "clusters": {"workload": "cluster creation (create_clusters.py, example dataset g22 configuration): "
                                        "one 1536x2048 frame per step -- ray generation + Voronoi routing of "
                                        "256 samples x 4 centroids per ray (YZ, margin 1.1) + per-expert AABB "
                                        "streaming; metric counts routed ray-samples", "frame": [1536, 2048],
                            "centroids": 4},
               "data": {"workload": f"TaskDataset construction (task_dataset.py _route_and_bin, nerf_runner.py "
                                    f"configuration: DDA routing, 1x5x5 cells): {a.data_rays} device-resident rays of "
                                    f"one region (images of the validation camera at downscale 0.25, pixel order) "
                                    f"routed, keep-filtered, stably binned per cell and copied to the host per step; "
                                    f"metric counts routed rays", "rays_per_gpu": a.data_rays}}[a.workload]
        cfg.update({"samples_per_ray": S, "parallelism": f"ray-sharded x{world}"})
        if a.workload == "c3" and a.diag_multi_last:
            cfg["plan"] = {"multi_expert_rays_last": True, "multi_expert_fraction": round(multi_frac, 4)}
        diag = {k: v for k, v in (("shared_table", a.diag_shared_table), ("pixel_order", a.diag_pixel_order),
                                  ("expert_only_order", a.diag_expert_only_order),
                                  ("multi_expert_rays_last", a.diag_multi_last),
                                  ("expert_box", a.diag_expert_box != "own" and a.diag_expert_box)) if v}
        if diag:        # a diagnostic run: not the workload's real render, never a headline line
            cfg["diagnostic"] = diag
        line = {
            "metric": "ray-samples/sec + PSNR, 4096 rays×256 samples, 1/2/4/8 MI355X",
            "value": round(value, 1), "unit": "rays/s" if a.workload == "data" else "ray-samples/s", "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
            "ms_per_step": round(ms_per_step, 4), "higher_is_better": True,
            "scaling": "strong" if (a.workload == "c4" or (a.workload == "c5" and a.c5_scaling == "strong"))
                       else "weak", "vs_baseline": None,
            "dtype": "f32", "data": "synthetic (formula-filled hash table, seeded MLP init; rays from the "
                                    "reference's validation camera geometry)",
            "config": cfg,
            "roofline": roofline,
            "cpu_baseline": cpu,
            "psnr_vs_cpu_path_db": None if psnr is None else round(psnr, 2),
            "rgb_max_abs_err_vs_cpu_path": maxerr,
        }
        if a.workload == "c2" and a.tau > 0:
            with torch.no_grad():
                ref0, _, _, acc0 = render_rays(model, rays, ray_samples=S, bg_color_default="white")
            line["early_termination"] = {
                "tau": a.tau, "max_abs_rgb_err_vs_tau0": float((out[0] - ref0).abs().max()),
                "rays_reaching_tau_frac": float(((1.0 - acc0) < a.tau).float().mean()),
                "bound": "2 * tau (the composite drops at most the remaining transmittance)",
                "note": "wavefront-level prefix product over each 32-sample tile; a ray stops at T < tau"}
        if a.workload == "c5":
            line["val_psnr_db"] = {"before": round(psnr_before, 3), "after": round(psnr_after, 3),
                                   "steps_adapted": int(a.warmup + a.steps + (5 if routed is not None else 0)), "val_rays": int(val_rays.shape[0]),
                                   "note": "linear-space PSNR (runtime_adapt.py:152-157) on held-out rays against a "
                                           "different 8-expert model's render (synthetic target)"}
            line["experts_hit_per_step"] = experts_hit
            if ep is not None:
                ep.flush()
                live = int(ep.seg[ep.K + 1: 2 * ep.K + 1].sum())
                line["exchange"] = {"bytes_sent_per_step_per_rank": ep.exchange_bytes(),
                                    "live_pair_bytes_per_step_per_rank": 56 * live + 8 * ep.K,
                                    "capacity_per_expert": ep.caps, "overflow_reruns": ep.overflows,
                                    "recaptures": ep.recaptures,
                                    "note": "sent = 8 B counts + 24 B record + 16 B result + 16 B gradient per pair "
                                            "slot at the step's capacities; live = the same for the routed pairs"}
        if a.workload == "c4":
            line["psnr_vs_synthetic_gt_db"] = round(float(out[3]), 4)
            if a.layout == "expert":
                # the owner kernel as ONE rank of the 8-GPU layout runs it (tools/ep_owner_rank.py: the records of
                # the busiest rank, one 128 MiB table resident), timed and counter-profiled on one GPU
                # the records in the order this run's renderer lays them out (depth tiles unless ACN_EP_TILE=0)
                from adaptive_city_nerf_amd import expert_parallel as _ep
                tile = int(os.environ.get("ACN_EP_TILE", _ep.EP_TILE_RAYS))
                src = (("r06_ep_owner_ranks_tiled.jsonl", "r06_pmc_ep_owner_rank2_tiled.json",
                        "r06_rocprof_ep_owner_rank2_tiled_kernel_stats.csv") if tile else
                       ("r06_ep_owner_ranks_bands.jsonl", "r06_pmc_ep_owner_rank2.json",
                        "r06_rocprof_ep_owner_rank2_kernel_stats.csv"))
                try:
                    pr = json.loads((REPO / "profiles" / src[1]).read_text())
                    ranks = [json.loads(l) for l in (REPO / "profiles" / src[0]).read_text()
                             .splitlines() if l.strip()]
                    busy = max((r for r in ranks if r.get("records")), key=lambda r: r["records"])
                    alg = pr["bytes_algorithmic_per_launch"]
                    ms = pr["rocprof_avg_ns"] / 1e6
                    line["per_rank_owner"] = {
                        "what": "ep_field_kernel of the busiest rank of the 8-GPU one-expert-per-GPU layout (expert "
                                f"{busy['rank_expert']}: {busy['records']} records of this frame; per-rank record "
                                f"counts {[r.get('records', 0) for r in ranks]})",
                        "record_order": f"depth tiles of {tile} rays" if tile else "sample order",
                        "kernel_ms_events": busy["kernel_ms"], "kernel_ms_rocprof": round(ms, 4),
                        "roofline": {"bound": "hbm", "achieved": round(alg / (ms * 1e-3) / 1e9, 1),
                                     "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                     "frac": round(alg / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                                     "traffic": pr["hbm_bytes_per_launch"], "bytes_per_record": 1064,
                                     "bytes_algorithmic_per_launch": alg,
                                     "l2_misses_per_record": round(pr["derived"]["l2_misses_per_sample"], 2)},
                        "source": ", ".join("profiles/" + f for f in src)}
                except Exception:
                    pass
            if a.layout == "expert" and ep_stats:
                line["exchange"] = {"bytes_sent_per_frame_per_rank": int(ep_stats["sent"]),
                                    "live_pair_bytes_per_frame_per_rank": int(ep_stats["live"]),
                                    "batches": int(ep_stats["batches"]),
                                    "note": "planned exchange (acn_routed_count_batches + one all-gather and one "
                                            "host read per frame): 24 B record out + 16 B result back per routed "
                                            "pair, no padding slot; rank 0's figures"}
        if a.workload in ("c5", "meta"):
            line["mlp_precision"] = a.mlp_precision
            if a.mlp_precision == "amp":
                line["dtype"] = "f16 MLP products / f32 accumulate (use_amp), f32 elsewhere"
                amp = getattr(routed, "amp", None) if a.workload == "c5" else None
                if amp is not None:
                    line["amp_scaler"] = amp.state_dict()
                if a.workload == "meta" and meta_scaler is not None:
                    line["amp_scaler"] = meta_scaler.state_dict()
        print(json.dumps(line))
    if world > 1:
        # release every graph that captured an RCCL collective (--ep-graph), then destroy the group, bounded:
        # RCCL's teardown waits for such graphs
        from adaptive_city_nerf_amd.expert_parallel import shutdown
        if not shutdown(timeout=120.0):
            print(f"bench.py rank {rank}: destroy_process_group did not return within 120 s", file=sys.stderr,
                  flush=True)
            sys.stdout.flush()
            os._exit(0)


if __name__ == "__main__":
    main()
