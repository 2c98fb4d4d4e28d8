#!/bin/bash
# Training-path MLP kernels: parity tests (fused vs composed, training / meta fixtures, graph replay)
# then the C5 and meta-training bench lines.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_mlp_train_gpu.py tests/test_train.py tests/test_meta_gpu.py tests/test_graph_gpu.py tests/test_module_api.py -m gpu -v --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_mlp.log 2>&1
echo "pytest rc=$?"
timeout -k 10 300 python bench.py --workload c5 --cpu-seconds 3 > gpurun_out/bench_c5m.json 2> gpurun_out/bench_c5m.err; echo "c5 rc=$?"
timeout -k 10 400 python bench.py --workload meta --steps 5 --warmup 2 --cpu-seconds 3 > gpurun_out/bench_metam.json 2> gpurun_out/bench_metam.err; echo "meta rc=$?"
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_mlp" -o run -- python "$GRAFT_REPO_ROOT/bench.py" --workload c5 --steps 20 --warmup 3 --cpu-seconds 0 > "$GRAFT_REPO_ROOT/gpurun_out/prof_mlp.log" 2>&1; echo "prof rc=$?"
