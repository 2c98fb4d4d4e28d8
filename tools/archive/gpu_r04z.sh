#!/bin/bash
# ray_order_kernel phase costs on the C2 batch: loads only (diag 3), + mean direction / coordinates (diag 2),
# fixed range instead of the bounding-box reduction (diag 1), full kernel (base)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04z; mkdir -p $O
for v in base odiag3 odiag2 odiag1; do
  if [ $v = base ]; then unset ACNERF_LIB; else export ACNERF_LIB=$PWD/build_variants/libacnerf_$v.so; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p_$v -o run -- python3 bench.py --steps 50 --no-cpu-baseline > $O/c2_$v.json 2>/dev/null || exit 1
  f=$(find $O/p_$v -name '*kernel_stats.csv' | head -1)
  python - "$f" "$v" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "ray_order" in r["Name"] or "render_kernel" in r["Name"]:
        print(sys.argv[2], r["Name"][:40], r["Calls"], r["AverageNs"])
PY
  find $O/p_$v -type f ! -name '*kernel_stats.csv' -delete
done
