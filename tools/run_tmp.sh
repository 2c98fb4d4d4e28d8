set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_loss_gpu.py tests/test_train.py tests/test_meta_gpu.py tests/test_graph_gpu.py tests/test_expert_parallel.py tests/test_mlp_train_gpu.py -m gpu -q --timeout 240 --timeout-method thread > gpurun_out/pt_loss.log 2>&1
echo pytest rc=$?
timeout -k 10 300 python -u bench.py --workload meta --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/meta_loss.json 2> gpurun_out/meta_loss.err &&
timeout -k 10 300 python -u bench.py --workload c5 --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/c5_loss.json 2> gpurun_out/c5_loss.err
echo rc=$?
