#!/bin/bash
# no-save training forward at four waves per SIMD: MLP / meta / train tests, MLP microbench, meta line
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03q
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_mlp_train_gpu.py tests/test_meta_gpu.py tests/test_train.py tests/test_graph_gpu.py -m gpu -q \
  --timeout 240 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|ERROR" $O/pytest.log | head -20; tail -2 $O/pytest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 200 python -u tools/micro/mlp_bench.py 2>&1 | grep -v amdgpu.ids | tail -3 || exit 1
timeout -k 10 400 python -u bench.py --workload meta --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_meta.json 2> $O/bench_meta.err || { echo "meta failed"; tail -5 $O/bench_meta.err; exit 3; }
cut -c150-260 $O/bench_meta.json
