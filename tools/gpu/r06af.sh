#!/bin/bash
# round 6: render_ws_kernel deriving the visiting order in its prologue (no ray_order_kernel launch) against the
# two-kernel form (noself) -- ws / ordered-render tests, C2 A/B, kernel summary of the default
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06af; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests/test_render_ws.py tests/test_gpu_kernels.py tests/test_module_api.py > $O/tests.txt 2>&1 || exit 1
for rep in 1 2; do
  for v in default noself; do
    if [ $v = default ]; then unset ACNERF_LIB; else export ACNERF_LIB=build_variants/libacnerf_$v.so; fi
    timeout -k 10 200 python -u bench.py --workload c2 --no-cpu-baseline > $O/c2_${v}_$rep.json 2> $O/c2_${v}_$rep.err || exit 2
  done
done
unset ACNERF_LIB
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c2 -o run -- python3 bench.py --no-cpu-baseline > $O/prof_c2.log 2>&1 || exit 3
find $O/prof_c2 -type f ! -name '*kernel_stats.csv' -delete
