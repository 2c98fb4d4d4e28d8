#!/bin/bash
# C5 kernel trace (per dispatch) to list one replayed step's launches and gaps
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04av; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o run -- python3 bench.py --workload c5 --steps 10 --warmup 3 --no-cpu-baseline > $O/c5.json 2>$O/c5.err || { tail -3 $O/c5.err; exit 1; }
f=$(find $O/trace -name '*kernel_trace.csv' | head -1); cp $f $O/c5_kernel_trace.csv
find $O/trace -type f ! -name '*kernel_trace.csv' -delete
wc -l $O/c5_kernel_trace.csv
