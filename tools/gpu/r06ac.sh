#!/bin/bash
# round 6: 16-ray rounds in render_wss_kernel (S <= 128) against 8-ray rounds -- routed tests per variant, C4-S96 A/B
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06ac; mkdir -p $O
for v in wss16 wss16r16; do
  ACNERF_LIB=build_variants/libacnerf_$v.so timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests/test_k8.py > $O/tests_$v.txt 2>&1 || exit 1
done
for rep in 1 2; do
  for v in wss8b wss16 wss16r16; do
    ACNERF_LIB=build_variants/libacnerf_$v.so timeout -k 10 300 python -u bench.py --workload c4 --samples 96 --steps 5 --no-cpu-baseline > $O/c4s96_${v}_$rep.json 2> $O/c4s96_${v}_$rep.err || exit 2
  done
done
