#!/bin/bash
# round 6: 8-ray depth tiles as the render_ws_kernel default -- full GPU suite + smoke, C2 bench (with CPU
# baseline), its kernel summary and counter passes
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06z; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_suite.txt 2>&1 || exit 1
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || exit 2
timeout -k 10 400 python -u bench.py > $O/bench_c2.json 2> $O/bench_c2.err || exit 3
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c2 -o run -- python3 bench.py --no-cpu-baseline > $O/prof_c2.log 2>&1 || exit 4
find $O/prof_c2 -type f ! -name '*kernel_stats.csv' -delete
timeout -k 10 600 bash tools/pmc_r04.sh r06z_c2 --workload c2 --no-cpu-baseline > $O/pmc_c2.log 2>&1 || exit 5
