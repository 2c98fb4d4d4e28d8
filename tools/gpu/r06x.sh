#!/bin/bash
# round 6: depth tiles in render_ws_kernel (ACN_WS_DTILE=1: a tile = the round's 16 rays at 2 samples) against
# the same build with ray tiles -- bitwise test of the ws render, C2 A/B with kernel stats
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06x; mkdir -p $O
ACNERF_LIB=build_variants/libacnerf_wsdt.so timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests/test_render_ws.py > $O/ws_tests_dt.txt 2>&1 || exit 1
for rep in 1 2; do
  for v in wsref wsdt; do
    ACNERF_LIB=build_variants/libacnerf_$v.so timeout -k 10 200 python -u bench.py --workload c2 --no-cpu-baseline > $O/c2_${v}_$rep.json 2> $O/c2_${v}_$rep.err || exit 2
  done
done
ACNERF_LIB=build_variants/libacnerf_wsdt.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_dt -o run -- python3 bench.py --no-cpu-baseline > $O/prof_dt.log 2>&1 || exit 3
find $O/prof_dt -type f ! -name '*kernel_stats.csv' -delete
