#!/bin/bash
# A/B the build_variants/*.so on the bench workload (each variant in its own process, own time limit).
# Usage (on the GPU box): [BENCH_ARGS="--workload c3"] tools/ab_variants.sh OUTFILE name1 name2 ...
set -o pipefail
OUT=$1; shift
mkdir -p gpurun_out
: > $OUT
for v in "$@"; do
  lib=adaptive_city_nerf_amd/libacnerf.so; [ "$v" = base ] || lib=build_variants/libacnerf_$v.so
  ACNERF_LIB=$lib timeout -k 10 120 python bench.py --steps 50 --warmup 5 --cpu-seconds 0.3 $BENCH_ARGS \
      > gpurun_out/ab_$v.json 2> gpurun_out/ab_$v.err || { echo "variant $v failed"; exit 1; }
  python - "$v" >> $OUT <<'PY'
import json, sys
v = sys.argv[1]
d = json.loads(open(f"gpurun_out/ab_{v}.json").read().strip().splitlines()[-1])
print(f"{v:10s} value={d['value']:.4e} kernel_ms={d['roofline']['kernel_ms']:.4f} frac={d['roofline']['frac']:.3f} "
      f"psnr={d['psnr_vs_cpu_path_db']} maxerr={d['rgb_max_abs_err_vs_cpu_path']}")
PY
done
cat $OUT
