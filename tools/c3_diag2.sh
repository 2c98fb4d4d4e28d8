#!/bin/bash
# C3 / C4 A/B of render variants (GPU box): tools/c3_diag2.sh variant...
set -o pipefail
mkdir -p gpurun_out
OUT=gpurun_out/c3_diag2.txt; : > $OUT
run() {  # name lib args...
  local name=$1 lib=$2; shift 2
  ACNERF_LIB=$lib timeout -k 10 120 python bench.py --steps 50 --warmup 5 --no-cpu-baseline "$@" > gpurun_out/c3d_$name.json 2> gpurun_out/c3d_$name.err || { echo "$name failed"; exit 1; }
  python -c "import json,sys; d=json.loads(open('gpurun_out/c3d_$name.json').read().strip().splitlines()[-1]); print(f\"$name {d['value']:.4e} kernel_ms={d['roofline']['kernel_ms']:.4f}\")" >> $OUT
}
for v in base "$@"; do
  L=adaptive_city_nerf_amd/libacnerf.so; [ $v = base ] || L=build_variants/libacnerf_$v.so
  run c3_$v $L --workload c3 && run c4_$v $L --workload c4 --steps 10 --warmup 2 \
    && run c4s96_$v $L --workload c4 --samples 96 --steps 10 --warmup 2 || exit 1
done
cat $OUT
