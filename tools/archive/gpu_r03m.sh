#!/bin/bash
# segment-mapped Adam unrolled + render_rays host-path caches: tests, C5 / C2 / C3 lines, C3 host time
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03m
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_train.py tests/test_module_api.py tests/test_k8.py tests/test_gpu_kernels.py tests/test_graph_gpu.py -m gpu -q \
  --timeout 240 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|ERROR" $O/pytest.log | head -20; tail -2 $O/pytest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 120 python -u tools/dbg/c3_host.py 2>&1 | grep -v amdgpu.ids | tail -2 || exit 1
b() { n=$1; shift; timeout -k 10 400 python -u bench.py "$@" > $O/bench_$n.json 2> $O/bench_$n.err || { echo "bench $n failed"; tail -5 $O/bench_$n.err; exit 3; }; echo "$n: $(cut -c150-260 $O/bench_$n.json)"; }
b c5 --workload c5 --no-cpu-baseline
b c2 --steps 20 --no-cpu-baseline
b c3 --workload c3 --no-cpu-baseline
