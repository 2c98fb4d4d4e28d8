#!/bin/bash
# Training-path GPU session: training parity tests, C5 + meta bench lines, rocprof of the meta step.
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-train}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_train.py tests/test_meta_gpu.py tests/test_gpu_kernels.py -v --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_$TAG.log 2>&1 \
&& timeout -k 10 300 python bench.py --workload c5 > gpurun_out/bench_c5_$TAG.json 2> gpurun_out/bench_c5_$TAG.err \
&& timeout -k 10 400 python bench.py --workload meta --steps 3 --warmup 1 --cpu-seconds 10 > gpurun_out/bench_meta_$TAG.json 2> gpurun_out/bench_meta_$TAG.err \
&& timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_meta_$TAG -o run -- python3 bench.py --workload meta --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/prof_meta_$TAG.log 2>&1
echo "gpu_train exit=$?"
