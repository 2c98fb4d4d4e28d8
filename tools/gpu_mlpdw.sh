#!/bin/bash
# Fused MLP backward session: training-path parity tests, then C5 + meta bench lines.
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-dw}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_sampler_gpu.py tests/test_mlp_train_gpu.py tests/test_train.py tests/test_meta_gpu.py tests/test_graph_gpu.py -v -x --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_$TAG.log 2>&1 \
&& timeout -k 10 300 python bench.py --workload c5 --no-cpu-baseline > gpurun_out/bench_c5_$TAG.json 2> gpurun_out/bench_c5_$TAG.err \
&& timeout -k 10 300 python bench.py --workload meta --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench_meta_$TAG.json 2> gpurun_out/bench_meta_$TAG.err
echo "gpu_mlpdw exit=$?"
