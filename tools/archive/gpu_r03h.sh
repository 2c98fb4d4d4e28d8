#!/bin/bash
# split routed render (EXSEL fix): render tests + C3 / C4 / C4-S96 / C2 bench lines
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03h
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_k8.py tests/test_gpu_kernels.py tests/test_expert_parallel.py tests/test_module_api.py tests/test_parallel.py -m gpu -q \
  --timeout 240 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1; echo "pytest rc=$?"; grep -E "FAILED|ERROR" $O/pytest.log | head -20; tail -2 $O/pytest.log
for w in "c3" "c4" "c4 --samples 96" "c2"; do
  n=$(echo $w | tr -d ' -')
  timeout -k 10 300 python -u bench.py --workload $w --no-cpu-baseline > $O/bench_$n.json 2> $O/bench_$n.err || { echo "bench $w failed"; tail $O/bench_$n.err; exit 3; }
  cat $O/bench_$n.json
done
