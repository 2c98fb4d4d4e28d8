#!/bin/bash
# round 6: the final bench lines (default C2 with its CPU baseline, C3, C4-S96, C4-S96 --layout expert, C5, meta)
# and the rocprof kernel summary of the default bench command
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06r; mkdir -p $O
timeout -k 10 400 python -u bench.py > $O/bench_c2.json 2> $O/bench_c2.err || exit 1
timeout -k 10 200 python -u bench.py --workload c3 > $O/bench_c3.json 2> $O/bench_c3.err || exit 2
timeout -k 10 300 python -u bench.py --workload c4 --samples 96 --steps 5 > $O/bench_c4s96.json 2> $O/bench_c4s96.err || exit 3
timeout -k 10 300 python -u bench.py --workload c4 --samples 96 --steps 5 --layout expert --no-cpu-baseline > $O/bench_c4s96_expert.json 2> $O/bench_c4s96_expert.err || exit 4
timeout -k 10 300 python -u bench.py --workload c5 > $O/bench_c5.json 2> $O/bench_c5.err || exit 5
timeout -k 10 300 python -u bench.py --workload meta > $O/bench_meta.json 2> $O/bench_meta.err || exit 6
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c2 -o run -- python3 bench.py --no-cpu-baseline > $O/prof_c2.log 2>&1 || exit 7
find $O/prof_c2 -type f ! -name '*kernel_stats.csv' -delete
