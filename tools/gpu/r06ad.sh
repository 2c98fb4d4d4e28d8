#!/bin/bash
# round 6: (1) the default build's routed rounds (16-ray rounds up to S = 128): routed tests, C3 / C4-S96 / C4 lines;
# (2) render_ws_kernel composite overlap (wsov) against the default: ws tests, C2 A/B
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06ad; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests/test_k8.py tests/test_parallel.py tests/test_batch_independence.py > $O/routed_tests.txt 2>&1 || exit 1
ACNERF_LIB=build_variants/libacnerf_wsov.so timeout -k 10 300 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread tests/test_render_ws.py > $O/ws_tests_wsov.txt 2>&1 || exit 2
timeout -k 10 200 python -u bench.py --workload c3 --no-cpu-baseline > $O/c3.json 2> $O/c3.err || exit 3
timeout -k 10 300 python -u bench.py --workload c4 --samples 96 --steps 5 --no-cpu-baseline > $O/c4s96.json 2> $O/c4s96.err || exit 3
timeout -k 10 300 python -u bench.py --workload c4 --steps 3 --no-cpu-baseline > $O/c4.json 2> $O/c4.err || exit 3
for rep in 1 2; do
  for v in default wsov; do
    if [ $v = default ]; then unset ACNERF_LIB; else export ACNERF_LIB=build_variants/libacnerf_$v.so; fi
    timeout -k 10 200 python -u bench.py --workload c2 --no-cpu-baseline > $O/c2_${v}_$rep.json 2> $O/c2_${v}_$rep.err || exit 4
  done
done
unset ACNERF_LIB
