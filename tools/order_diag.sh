#!/bin/bash
# ray_order_kernel cost: rocprof kernel stats of the C2 bench (base build and any build_variants given,
# e.g. tools/build_variants.sh od1:render.hip:"-DACN_ORDER_DIAG=1" ... ; then tools/order_diag.sh od1 od2 od3)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/order_diag.txt
for v in base "$@"; do
  L=adaptive_city_nerf_amd/libacnerf.so; [ $v = base ] || L=build_variants/libacnerf_$v.so
  ACNERF_LIB=$L timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pod_$v -o run -- python3 bench.py --steps 100 --warmup 5 --no-cpu-baseline > gpurun_out/pod_$v.log 2>&1 || exit 1
  python - $v >> gpurun_out/order_diag.txt <<'PY'
import csv, sys
v = sys.argv[1]
for r in csv.DictReader(open(f"gpurun_out/pod_{v}/run_kernel_stats.csv")):
    if "ray_order" in r["Name"] or "render_kernel" in r["Name"]:
        print(v, r["Name"][:40], r["AverageNs"], r["MinNs"])
PY
done
cat gpurun_out/order_diag.txt
