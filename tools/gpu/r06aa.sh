#!/bin/bash
# round 6: routed render in depth tiles (render_wss_kernel) -- routed-render tests on the default build, then
# C3 / C4-S96 A/B against render_slots_kernel (nowss) and 4- / 2-ray tiles
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06aa; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests/test_k8.py tests/test_render_ws.py tests/test_parallel.py tests/test_batch_independence.py > $O/tests.txt 2>&1 || exit 1
for rep in 1 2; do
  for v in nowss default wss4 wss2; do
    if [ $v = default ]; then unset ACNERF_LIB; else export ACNERF_LIB=build_variants/libacnerf_$v.so; fi
    timeout -k 10 200 python -u bench.py --workload c3 --no-cpu-baseline > $O/c3_${v}_$rep.json 2> $O/c3_${v}_$rep.err || exit 2
    timeout -k 10 300 python -u bench.py --workload c4 --samples 96 --steps 5 --no-cpu-baseline > $O/c4s96_${v}_$rep.json 2> $O/c4s96_${v}_$rep.err || exit 3
  done
done
unset ACNERF_LIB
