#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03l
mkdir -p $O
timeout -k 10 120 python -u tools/dbg/c3_host.py 2>&1 | grep -v amdgpu.ids | tail -3 || exit 1
timeout -k 10 400 python -u bench.py --workload c5 > $O/bench_c5.json 2> $O/bench_c5.err || { echo "bench c5 failed"; tail -5 $O/bench_c5.err; exit 3; }
cut -c1-300 $O/bench_c5.json
