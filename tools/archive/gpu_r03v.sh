#!/bin/bash
# producer / consumer fused MLP backward: tests (bounded), then A/B timing and the meta line
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03v
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_mlp_train_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_mlp.log 2>&1; rc=$?
echo "mlp tests rc=$rc"; tail -2 $O/pytest_mlp.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_meta_gpu.py tests/test_train.py tests/test_graph_gpu.py -m gpu -q --timeout 240 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "FAILED|ERROR" $O/pytest.log | head; tail -2 $O/pytest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
echo "== pc"; timeout -k 10 200 python -u tools/micro/mlp_bench.py 2>&1 | grep -v amdgpu.ids | tail -2 || exit 1
echo "== no pc"; ACNERF_LIB=build_variants/libacnerf_nopc.so timeout -k 10 200 python -u tools/micro/mlp_bench.py 2>&1 | grep -v amdgpu.ids | tail -2 || exit 1
timeout -k 10 400 python -u bench.py --workload meta --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_meta.json 2> $O/bench_meta.err || { echo "meta failed"; tail -5 $O/bench_meta.err; exit 3; }
cut -c150-260 $O/bench_meta.json
