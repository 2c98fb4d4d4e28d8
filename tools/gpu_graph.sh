set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_graph_gpu.py tests/test_train.py -v -m gpu --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_graph.log 2>&1
echo "pytest rc=$?"
timeout -k 10 300 python bench.py --workload c5 --cpu-seconds 3 > gpurun_out/bench_c5g.json 2> gpurun_out/bench_c5g.err; echo "bench graph rc=$?"
timeout -k 10 300 python bench.py --workload c5 --no-graph --no-cpu-baseline > gpurun_out/bench_c5e.json 2> gpurun_out/bench_c5e.err; echo "bench eager rc=$?"
