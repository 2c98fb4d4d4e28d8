"""Gather-only ceiling of the fused render's hash-table access (developer tool; VERDICT r02 "Next" 1).

python tools/micro/hash_gather.py [--out gpurun_out/hash_gather.json]

Builds tools/micro/hash_gather.hip into tools/micro/build/libhash_gather.so (hipcc, gfx950) if needed, then on
cuda:0, for the C2 workload (bench.py: 4096 rays x 256 samples of validation camera 0, one expert, the same
formula-filled 128 MiB table):
  * times the product render (render_rays, eval) the way bench.py does (random ray order + ray_order_kernel),
    and on the same rays in pixel order with the reordering off;
  * times gather_kernel (hash_gather.hip: the render's hash access and nothing else) over the SAME sample
    points (the eval t-values of acn_sample_stratified, unit-box points of the expert) in pixel order,
    sweeping the levels in flight (1-4), the workgroups per CU (1-4, i.e. 4-16 waves) and XCD bands on / off;
  * and over uniformly random points (no locality between samples) for comparison.
Algorithmic bytes are SURVEY §8(d)'s 1024 B per sample (16 levels x 8 corners x 8 B).  The best gather-only
time on the C2 points is the ceiling the render's gathers can reach (the render additionally runs the MLP and
the compositing in the same waves)."""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import subprocess
import sys
from pathlib import Path

import numpy as np
import torch

HERE = Path(__file__).resolve().parent
REPO = HERE.parents[1]
sys.path.insert(0, str(REPO))
LIB = HERE / "build" / "libhash_gather.so"


def build() -> None:
    src = HERE / "hash_gather.hip"
    deps = [src, REPO / "adaptive_city_nerf_amd" / "csrc" / "acn_device.h"]
    if LIB.exists() and LIB.stat().st_mtime >= max(d.stat().st_mtime for d in deps):
        return
    LIB.parent.mkdir(exist_ok=True)
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off",
                    "-mcode-object-version=5", "-shared", "-o", str(LIB), str(src)], check=True)


def time_ms(fn, reps: int) -> float:
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=str(REPO / "gpurun_out" / "hash_gather.json"))
    ap.add_argument("--reps", type=int, default=100)
    a = ap.parse_args()
    build()
    import bench
    from adaptive_city_nerf_amd import ops, render_rays
    from adaptive_city_nerf_amd.ray_rendering import ENC_EPS
    dev = torch.device("cuda", 0)
    model, gbox, scene, sc = bench.build_model(dev, 1)
    sub = model.submodules[0]
    enc = sub.xyz_encoder
    S, N = 256, 4096
    rays = bench.make_rays(scene, gbox, dev, N, 1234)
    rays_px = bench.make_rays(scene, gbox, dev, N, 1234, pixel_order=True)
    res = (C.c_float * 16)(*[float(v) for v in enc._res_host])
    table = enc.hash_table.detach().contiguous()
    lib = C.CDLL(str(LIB))
    lib.hg_launch.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                              C.c_void_p, C.c_void_p]
    ncu = torch.cuda.get_device_properties(dev).multi_processor_count
    M = N * S
    alg_bytes = 1024.0 * M
    out = torch.empty(M, 2, device=dev, dtype=torch.float32)
    mn, ext = sub._host_box()
    _, x01_px, _ = ops.sample_stratified(rays_px, S, None, mn, ext, float(ENC_EPS))
    x01_uni = torch.rand(M, 3, device=dev, generator=torch.Generator(dev).manual_seed(5)).clamp_(1e-6, 1 - 1e-6)
    result = {"workload": "C2 (bench.py): 4096 rays x 256 samples, one expert, L=16 x 2^20 x F=2 fp32 table (128 MiB)",
              "alg_bytes_per_launch": alg_bytes, "cus": ncu, "reps": a.reps}

    with torch.no_grad():
        def rend(r, reorder):
            ops.REORDER = reorder
            return render_rays(model, r, ray_samples=S, bg_color_default="white", _want_weights=True)
        t_render = time_ms(lambda: rend(rays, True), a.reps)
        t_render_px = time_ms(lambda: rend(rays_px, False), a.reps)
        ops.REORDER = True
    result["render_ms"] = {"bench_random_order_reordered": t_render, "pixel_order_no_reorder": t_render_px}

    sweeps = []
    stream = torch.cuda.current_stream(dev).cuda_stream
    for name, pts in (("c2_points_pixel_order", x01_px), ("uniform_random_points", x01_uni)):
        for band in (1, 0):
            for depth in (1, 2, 3, 4):
                for bpc in (1, 2, 3, 4):
                    blocks = ((ncu * bpc + 7) // 8) * 8

                    def go():
                        rc = lib.hg_launch(pts.data_ptr(), table.data_ptr(), C.cast(res, C.c_void_p), enc.log2_hashmap_size,
                                           N, S, depth, blocks, band, out.data_ptr(), C.c_void_p(stream))
                        assert rc == 0, rc
                    ms = time_ms(go, a.reps)
                    sweeps.append({"points": name, "band": band, "depth": depth, "waves_per_cu": 4 * bpc, "ms": round(ms, 4),
                                   "alg_gbs": round(alg_bytes / (ms * 1e-3) / 1e9, 1)})
                    print(json.dumps(sweeps[-1]), flush=True)
    best = min((s for s in sweeps if s["points"] == "c2_points_pixel_order"), key=lambda s: s["ms"])
    best_u = min((s for s in sweeps if s["points"] == "uniform_random_points"), key=lambda s: s["ms"])
    result["sweeps"] = sweeps
    result["ceiling"] = {"config": best, "alg_gbs": best["alg_gbs"],
                         "render_frac_of_ceiling": round(best["ms"] / t_render, 4),
                         "render_px_frac_of_ceiling": round(best["ms"] / t_render_px, 4)}
    result["uniform_best"] = best_u
    Path(a.out).parent.mkdir(parents=True, exist_ok=True)
    Path(a.out).write_text(json.dumps(result, indent=1))
    print(json.dumps({k: result[k] for k in ("render_ms", "ceiling", "uniform_best")}))


if __name__ == "__main__":
    main()
