#!/bin/bash
# Cluster-creation GPU session: parity tests, bench line, rocprof kernel stats.
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-clusters}
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_cluster_gpu.py -v -s --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_$TAG.log 2>&1 \
&& timeout -k 10 300 python bench.py --workload clusters --cpu-seconds 10 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err \
&& timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- python3 bench.py --workload clusters --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/prof_$TAG.log 2>&1
echo "gpu_clusters exit=$?"
