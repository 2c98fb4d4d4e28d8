#!/bin/bash
# round 5: counter passes for C2 (render_ws_kernel) on the final render build, and one C5 kernel trace
# (the per-step launch sequence of the replayed adaptation step, for the glue fusion)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05r; mkdir -p $O
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/c5trace -o run -- python3 bench.py --workload c5 --steps 4 --warmup 3 --no-cpu-baseline > $O/c5trace.log 2>&1 || exit 1
find $O/c5trace -type f ! -name '*kernel_trace.csv' -delete
bash tools/pmc_r04.sh c2_r05 --steps 20 --no-cpu-baseline || exit 2
