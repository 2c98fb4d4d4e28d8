#!/bin/bash
# Meta-training GPU session: bench line + rocprof kernel stats.
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-meta}
mkdir -p gpurun_out
timeout -k 10 400 python bench.py --workload meta --steps 3 --warmup 1 --cpu-seconds 10 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err \
&& timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- python3 bench.py --workload meta --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/prof_$TAG.log 2>&1
echo "gpu_meta exit=$?"
