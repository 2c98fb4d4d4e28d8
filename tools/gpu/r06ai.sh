#!/bin/bash
# round 6 (resumed session): the current build (ACN_HASH_DEPTH 3 default) -- full GPU suite + smoke, C2 / C3 /
# C4-S96 / C5 / meta bench lines, the C2 kernel summary
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06ai; mkdir -p $O
unset ACNERF_LIB
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_suite.txt 2>&1 || exit 1
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || exit 2
timeout -k 10 400 python -u bench.py > $O/bench_c2.json 2> $O/bench_c2.err || exit 3
timeout -k 10 200 python -u bench.py --workload c3 --no-cpu-baseline > $O/bench_c3.json 2> $O/bench_c3.err || exit 4
timeout -k 10 300 python -u bench.py --workload c4 --samples 96 --steps 5 --no-cpu-baseline > $O/bench_c4s96.json 2> $O/bench_c4s96.err || exit 5
timeout -k 10 300 python -u bench.py --workload c5 --no-cpu-baseline > $O/bench_c5.json 2> $O/bench_c5.err || exit 7
timeout -k 10 300 python -u bench.py --workload meta --no-cpu-baseline > $O/bench_meta.json 2> $O/bench_meta.err || exit 8
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c2 -o run -- python3 bench.py --no-cpu-baseline > $O/prof_c2.log 2>&1 || exit 9
find $O/prof_c2 -type f ! -name '*kernel_stats.csv' -delete
