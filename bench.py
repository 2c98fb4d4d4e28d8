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

import numpy as np
import torch
import torch.distributed as dist

REPO = Path(__file__).resolve().parent
sys.path.insert(0, str(REPO))

FLOP_PER_SAMPLE = 26880          # MLP MACs x 2: 32*64+64*64+64+64*15+31*64+64*64+64*3 = 13,440
BYTES_PER_SAMPLE = 1024.2        # algorithmic hash-table reads + amortised ray I/O
FP32_MFMA_PEAK_TFLOPS = 157.3    # MI355X_MICROARCH.md: FP32 matrix = vector peak (spec)
HBM_PEAK_GBS = 8000.0


def build_model(device, n_experts=1, seed=0, table_seed=100, table_scale=0.5):
    from adaptive_city_nerf_amd import MetaContainer, SceneBox
    from adaptive_city_nerf_amd.synthetic import formula_table
    scene = json.loads((REPO / "tests" / "golden" / "scene_drz_example.json").read_text())
    mask = "g11_grid_bm110_ss11" if n_experts == 1 else "g22_grid_bm110_ss11"
    sc = scene["masks"][mask]
    K = len(sc["centroids"])
    gbox = SceneBox(aabb=torch.tensor(sc["aabb_global"], dtype=torch.float32))
    boxes = [SceneBox(aabb=torch.tensor([sc["mins"][k], sc["maxs"][k]], dtype=torch.float32)) for k in range(K)]
    torch.manual_seed(seed)
    m = MetaContainer(num_submodules=K, centroids=torch.tensor(sc["centroids"]), aabb=gbox.aabb,
                      nerf_variant="instant", boundary_margin=min(max(1.0, 1.05), sc["boundary_margin"]),
                      cluster_2d=sc["cluster_2d"], use_bg_nerf=True, bg_hidden=32, occ_conf={"use_occ": False},
                      expert_box_list=boxes, hidden=64, sigma_depth=2, color_depth=2, dir_encoding="spherical",
                      color_hidden=64, use_sigmoid_rgb=True,
                      hash_enc_conf={"levels": 16, "features_per_level": 2, "log2_hashmap_size": 20,
                                     "max_res": 4096, "min_res": 16, "interpolation": "Linear"})
    with torch.no_grad():
        for k, sub in enumerate(m.submodules):
            sub.xyz_encoder.hash_table.copy_(torch.from_numpy(formula_table(16, 20, 2, table_seed + k, table_scale)))
    return m.to(device).eval(), gbox, scene, sc


def make_rays(scene, gbox, device, n_rays, seed):
    from adaptive_city_nerf_amd import ops
    cam = scene["val_cam0"]
    ds = 0.25
    H, W = int(round(cam["H"] * ds)), int(round(cam["W"] * ds))
    intr = (torch.tensor(cam["intrinsics"], dtype=torch.float32) * ds).tolist()
    psf = scene["pose_scale_factor"]
    rays, valid = ops.get_rays_image(H, W, *intr, torch.tensor(cam["c2w"]), gbox.aabb, device,
                                     near_far_override=(0.0 / psf, 100000 / psf))
    vi = torch.nonzero(valid).squeeze(1).cpu()
    g = torch.Generator().manual_seed(seed)
    sel = vi[torch.randperm(vi.numel(), generator=g)[:n_rays]]
    return rays[sel.to(device)].contiguous()


def cpu_baseline(model, sc, rays, S, gpu_rgb, min_seconds):
    """C oracle on the host cores over the same batch, repeated until >= min_seconds."""
    from oracle import oracle as O
    sub = model.submodules[0]
    w = {n: p.detach().cpu().numpy() for n, p in sub.meta_named_parameters()}
    e = O.Expert(w, sub.xyz_encoder.hash_table.detach().cpu().numpy(), np.array(sub.xyz_encoder._res_host, np.int32),
                 sub.scene_box.min.cpu().numpy(), sub.aabb_extent.cpu().numpy())
    bg = {f"bg_mlp.{k}": v.detach().cpu().numpy() for k, v in model.bg_mlp.state_dict().items()}
    r = rays.cpu().numpy()
    cores = O.max_threads()
    reps, t0 = 0, time.perf_counter()
    while True:
        orgb, _, _, _ = O.render_stratified(r, S, [e], np.array(sc["centroids"], np.float32), bm=model.boundary_margin,
                                            bg_mlp=bg, want_weights=False)
        reps += 1
        if time.perf_counter() - t0 >= min_seconds:
            break
    dt = time.perf_counter() - t0
    mse = float(np.mean((gpu_rgb.astype(np.float64) - orgb.astype(np.float64)) ** 2))
    psnr = float("inf") if mse == 0 else -10.0 * np.log10(mse)
    return {"value": r.shape[0] * S * reps / dt, "unit": "ray-samples/s", "cores": cores, "kind": "port",
            "sample": f"{reps} x ({r.shape[0]} rays x {S} samples) of the benchmark batch, C oracle "
                      f"(oracle/acn_oracle.c, OpenMP {cores} threads), {dt:.1f} s"}, psnr, float(np.sqrt(mse)), \
        float(np.max(np.abs(gpu_rgb - orgb)))


def load_traffic():
    p = REPO / "profiles" / "pmc_render_r01.json"
    if p.exists():
        try:
            return json.loads(p.read_text())
        except Exception:
            return None
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--rays", type=int, default=4096)
    ap.add_argument("--samples", type=int, default=256)
    ap.add_argument("--experts", type=int, default=1)
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    a = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    device = torch.device("cuda", local)
    torch.cuda.set_device(device)

    from adaptive_city_nerf_amd import ops, render_rays
    model, gbox, scene, sc = build_model(device, a.experts)
    rays = make_rays(scene, gbox, device, a.rays, 1234 + rank)
    S = a.samples

    def step():
        with torch.no_grad():
            return render_rays(model, rays, ray_samples=S, bg_color_default="white")

    for _ in range(a.warmup):
        out = step()
    torch.cuda.synchronize()
    ops.EVENT_HOOK = []
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        out = step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    kernel_ms = float(np.mean([e0.elapsed_time(e1) for e0, e1 in ops.EVENT_HOOK]))
    ops.EVENT_HOOK = None
    if world > 1:
        t = torch.tensor([dt, kernel_ms], device=device, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt, kernel_ms = float(t[0]), float(t[1])

    samples_per_step = a.rays * S
    value = world * samples_per_step * a.steps / dt
    ms_per_step = dt / a.steps * 1e3
    achieved = FLOP_PER_SAMPLE * samples_per_step / (kernel_ms * 1e-3) / 1e12
    tr = load_traffic()
    roofline = {"bound": "mfma", "achieved": round(achieved, 2), "peak": FP32_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s",
                "frac": round(achieved / FP32_MFMA_PEAK_TFLOPS, 4),
                "traffic": (tr or {}).get("hbm_bytes_per_launch"),
                "kernel": "render_kernel<1,1,0> (fused stratified render)", "kernel_ms": round(kernel_ms, 4),
                "hash_bytes_algorithmic_per_launch": int(BYTES_PER_SAMPLE * samples_per_step),
                "hash_gbs_algorithmic": round(BYTES_PER_SAMPLE * samples_per_step / (kernel_ms * 1e-3) / 1e9, 1)}

    cpu, psnr, rmse, maxerr = None, None, None, None
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        cpu, psnr, rmse, maxerr = cpu_baseline(model, sc, rays, S, out[0].cpu().numpy(), a.cpu_seconds)

    if rank == 0:
        line = {
            "metric": "ray-samples/sec + PSNR, 4096 rays×256 samples, 1/2/4/8 MI355X",
            "value": round(value, 1), "unit": "ray-samples/s", "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
            "ms_per_step": round(ms_per_step, 4), "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "f32", "data": "synthetic (formula-filled hash table, seeded MLP init; rays from the "
                                    "reference's validation camera geometry)",
            "config": {"workload": "C2: single Instant-NGP expert, 4096 rays x 256 samples per GPU, eval, fused "
                                   "render_rays", "rays_per_gpu": a.rays, "samples_per_ray": S,
                       "experts": a.experts, "parallelism": f"ray-sharded x{world}"},
            "roofline": roofline,
            "cpu_baseline": cpu,
            "psnr_vs_cpu_path_db": None if psnr is None else round(psnr, 2),
            "rgb_max_abs_err_vs_cpu_path": maxerr,
        }
        print(json.dumps(line))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
