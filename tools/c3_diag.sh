#!/bin/bash
# C3 diagnostics (GPU box): Infinity-Cache capacity (shared table) and batch order (pixel order, XCD bands).
set -o pipefail
mkdir -p gpurun_out
OUT=gpurun_out/c3_diag.txt; : > $OUT
run() {  # name lib args...
  local name=$1 lib=$2; shift 2
  ACNERF_LIB=$lib timeout -k 10 120 python bench.py --steps 50 --warmup 5 --no-cpu-baseline "$@" > gpurun_out/c3d_$name.json 2> gpurun_out/c3d_$name.err || { echo "$name failed"; exit 1; }
  python -c "import json,sys; d=json.loads(open('gpurun_out/c3d_$name.json').read().strip().splitlines()[-1]); print(f\"$name {d['value']:.4e} kernel_ms={d['roofline']['kernel_ms']:.4f}\")" >> $OUT
}
B=adaptive_city_nerf_amd/libacnerf.so
run c2 $B --workload c2 && run c3 $B --workload c3 && run c3_shared $B --workload c3 --diag-shared-table \
 && run c3_pix $B --workload c3 --diag-pixel-order && run c3_pix_band build_variants/libacnerf_band.so --workload c3 --diag-pixel-order \
 && run c3_pix_shared $B --workload c3 --diag-pixel-order --diag-shared-table
cat $OUT
