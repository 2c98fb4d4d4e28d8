"""A/B of the standalone hash-grid forward's access shape (developer tool).

python tools/micro/hash_fwd.py [--out gpurun_out/hash_fwd.json]

Builds tools/micro/hash_fwd.hip (hipcc, gfx950) if needed, then on cuda:0 times three variants of the F = 2 linear
forward (plain 8 x dwordx2 gathers / x-pair 16-B blocks / x-pair + XCD level bands, see the .hip header) and the
product's acn_hashgrid_fwd over the same points of bench.py's C2 scene (one expert, 2^20-row levels):
  * 4096 rays x 96 samples in random ray order (the meta step's query/support batches are random rays, ray-major);
  * 4096 rays x 256 samples in pixel order.
Every variant's output must equal the product's bit for bit."""
from __future__ import annotations

import argparse
import ctypes as C
import json
import subprocess
import sys
from pathlib import Path

import torch

HERE = Path(__file__).resolve().parent
REPO = HERE.parents[1]
sys.path.insert(0, str(REPO))
LIB = HERE / "build" / "libhash_fwd.so"


def build() -> None:
    src = HERE / "hash_fwd.hip"
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
    ap.add_argument("--out", default=str(REPO / "gpurun_out" / "hash_fwd.json"))
    ap.add_argument("--reps", type=int, default=200)
    a = ap.parse_args()
    build()
    if not torch.cuda.is_available():
        print("built", LIB)
        return
    import bench
    from adaptive_city_nerf_amd import ops
    from adaptive_city_nerf_amd.ray_rendering import ENC_EPS
    dev = torch.device("cuda", 0)
    model, gbox, scene, sc = bench.build_model(dev, 1)
    sub = model.submodules[0]
    enc = sub.xyz_encoder
    table = enc.hash_table.detach().contiguous()
    res = torch.tensor([int(v) for v in enc._res_host], dtype=torch.int32)
    log2T = int(enc.log2_hashmap_size)
    mn, ext = sub._host_box()
    lib = C.CDLL(str(LIB))
    lib.hf_launch.argtypes = [C.c_int, C.c_void_p, C.c_int64, C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.c_void_p]
    stream = torch.cuda.current_stream(dev).cuda_stream
    result = {"table": f"L=16 x 2^{log2T} x F=2 fp32", "reps": a.reps, "cases": []}
    for name, S, px in (("random_rays_S96", 96, False), ("pixel_order_S256", 256, True)):
        rays = bench.make_rays(scene, gbox, dev, 4096, 1234, pixel_order=px)
        _, x01, _ = ops.sample_stratified(rays, S, None, mn, ext, float(ENC_EPS))
        x01 = x01.reshape(-1, 3).contiguous()
        M = x01.shape[0]
        box = {}

        def go_prod():
            box["o"] = ops.hashgrid_fwd(x01, table, enc._res_host, log2T, 2, 1)
        row = {"points": name, "M": M, "product_ms": round(time_ms(go_prod, a.reps), 4)}
        outs = {}
        for v, vn in ((0, "plain"), (1, "xpair"), (2, "band")):
            o = torch.empty(M, 32, device=dev)

            def go(v=v, o=o):
                rc = lib.hf_launch(v, x01.data_ptr(), M, table.data_ptr(), C.cast(res.data_ptr(), C.c_void_p), log2T,
                                   o.data_ptr(), C.c_void_p(stream))
                assert rc == 0, rc
            row[vn + "_ms"] = round(time_ms(go, a.reps), 4)
            outs[vn] = o
        for vn in ("xpair", "band"):
            row[vn + "_bitexact_vs_plain"] = bool(torch.equal(outs[vn], outs["plain"]))
        row["plain_bitexact_vs_product"] = bool(torch.equal(outs["plain"], box["o"].reshape(M, 32)))
        row["alg_gbs_plain"] = round(1024.0 * M / (row["plain_ms"] * 1e-3) / 1e9, 1)
        result["cases"].append(row)
        print(json.dumps(row), flush=True)
    Path(a.out).parent.mkdir(parents=True, exist_ok=True)
    Path(a.out).write_text(json.dumps(result, indent=1))


if __name__ == "__main__":
    main()
