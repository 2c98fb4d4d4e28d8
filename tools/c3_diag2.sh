#!/bin/bash
# C3 / C4 batch-order A/B (GPU box): expert-only vs (expert, direction cell) order, XCD bands in render_slots_kernel
set -o pipefail
mkdir -p gpurun_out
OUT=gpurun_out/c3_diag2.txt; : > $OUT
run() {  # name lib args...
  local name=$1 lib=$2; shift 2
  ACNERF_LIB=$lib timeout -k 10 120 python bench.py --steps 50 --warmup 5 --no-cpu-baseline "$@" > gpurun_out/c3d_$name.json 2> gpurun_out/c3d_$name.err || { echo "$name failed"; exit 1; }
  python -c "import json,sys; d=json.loads(open('gpurun_out/c3d_$name.json').read().strip().splitlines()[-1]); print(f\"$name {d['value']:.4e} kernel_ms={d['roofline']['kernel_ms']:.4f}\")" >> $OUT
}
B=adaptive_city_nerf_amd/libacnerf.so; V=build_variants/libacnerf_band.so
run c3_expertonly $B --workload c3 --diag-expert-only-order && run c3_cell $B --workload c3 \
 && run c3_expertonly_band $V --workload c3 --diag-expert-only-order && run c3_cell_band $V --workload c3 \
 && run c4 $B --workload c4 --steps 10 --warmup 2 && run c4_band $V --workload c4 --steps 10 --warmup 2 \
 && run c4s96 $B --workload c4 --samples 96 --steps 10 --warmup 2 && run c4s96_band $V --workload c4 --samples 96 --steps 10 --warmup 2
cat $OUT
