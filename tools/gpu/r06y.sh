#!/bin/bash
# round 6: rays per depth tile in render_ws_kernel (ACN_WS_DTILE = 16 / 8 / 4 / 2) against ray tiles (wsref):
# bitwise ws tests per variant, C2 A/B (two runs each, interleaved)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06y; mkdir -p $O
for v in wsdt16 wsdt8 wsdt4 wsdt2; do
  ACNERF_LIB=build_variants/libacnerf_$v.so timeout -k 10 300 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread tests/test_render_ws.py > $O/ws_tests_$v.txt 2>&1 || exit 1
done
for rep in 1 2; do
  for v in wsref wsdt16 wsdt8 wsdt4 wsdt2; do
    ACNERF_LIB=build_variants/libacnerf_$v.so timeout -k 10 200 python -u bench.py --workload c2 --no-cpu-baseline > $O/c2_${v}_$rep.json 2> $O/c2_${v}_$rep.err || exit 2
  done
done
