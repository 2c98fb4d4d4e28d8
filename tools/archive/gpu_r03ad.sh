#!/bin/bash
# final round-3 build: C5 bench line (with its CPU baseline) and rocprof summary
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03ad
mkdir -p $O
timeout -k 10 400 python -u bench.py --workload c5 > $O/bench_c5.json 2> $O/bench_c5.err || { echo "c5 failed"; tail -5 $O/bench_c5.err; exit 3; }
cut -c1-200 $O/bench_c5.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c5 -o run -- python3 bench.py --workload c5 --no-cpu-baseline > $O/prof_c5.log 2>&1 || { echo "prof c5 failed"; exit 4; }
find $O/prof_c5 -type f ! -name '*kernel_stats.csv' -delete
echo "r03ad done"
