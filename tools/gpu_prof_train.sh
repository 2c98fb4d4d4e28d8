#!/bin/bash
# Kernel-time profiles (stats CSVs only) of the meta-training and C5 workloads.
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-train}
mkdir -p gpurun_out
keep_stats() { find "$1" -type f ! -name '*kernel_stats.csv' -delete; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_meta_$TAG -o run -- python3 bench.py --workload meta --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof_meta_$TAG.log 2>&1 && keep_stats gpurun_out/prof_meta_$TAG \
&& timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c5_$TAG -o run -- python3 bench.py --workload c5 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/prof_c5_$TAG.log 2>&1 && keep_stats gpurun_out/prof_c5_$TAG
echo "gpu_prof_train exit=$?"
