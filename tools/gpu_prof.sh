#!/bin/bash
# rocprofv3 kernel stats of one bench workload: tools/gpu_prof.sh TAG "<bench args>"
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=$1
ARGS=$2
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- python3 bench.py $ARGS --no-cpu-baseline > gpurun_out/prof_$TAG.log 2>&1
rc=$?
echo "prof rc=$rc"
f=$(find gpurun_out/prof_$TAG -name "*kernel_stats.csv" | head -1)
[ -n "$f" ] && cp "$f" gpurun_out/prof_${TAG}_kernel_stats.csv
exit $rc
