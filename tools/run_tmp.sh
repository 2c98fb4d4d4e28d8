set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_expert_parallel.py tests/test_train.py tests/test_mlp_train_gpu.py tests/test_meta_gpu.py tests/test_graph_gpu.py tests/test_k8.py -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pt_nasm.log 2>&1
echo "pytest: $(tail -1 gpurun_out/pt_nasm.log)"
timeout -k 10 100 python -u tools/micro/mlp_bench.py > gpurun_out/mlpb_nasm.txt 2>&1
timeout -k 10 300 python -u bench.py --workload meta --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/meta_nasm.json 2> gpurun_out/meta_nasm.err
echo done
