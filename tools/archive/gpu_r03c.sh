#!/bin/bash
# round 3: drop-in training paths, sync-free expert-parallel step, split routed render: tests + bench lines
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03c
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests/test_train.py tests/test_meta_gpu.py tests/test_graph_gpu.py tests/test_loss_gpu.py \
  tests/test_expert_parallel.py tests/test_k8.py tests/test_gpu_kernels.py -m gpu -v \
  --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR" $O/pytest.log | grep -v PASSED | head -30
tail -3 $O/pytest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for w in "c3" "c4" "c2"; do
  timeout -k 10 300 python -u bench.py --workload $w --no-cpu-baseline > $O/bench_$w.json 2> $O/bench_$w.err || { echo "bench $w failed"; tail $O/bench_$w.err; exit 3; }
  cat $O/bench_$w.json
done
timeout -k 10 300 python -u bench.py --workload c5 --no-cpu-baseline > $O/bench_c5.json 2> $O/bench_c5.err || { echo "bench c5 failed"; tail $O/bench_c5.err; exit 4; }
cat $O/bench_c5.json
timeout -k 10 300 python -u bench.py --workload c5 --driver runtime_adapt --no-cpu-baseline > $O/bench_c5_ra.json 2> $O/bench_c5_ra.err || { echo "bench c5 ra failed"; tail $O/bench_c5_ra.err; exit 5; }
cat $O/bench_c5_ra.json
timeout -k 10 300 python -u bench.py --workload meta --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_meta.json 2> $O/bench_meta.err || { echo "bench meta failed"; tail $O/bench_meta.err; exit 6; }
cat $O/bench_meta.json
echo "r03c done"
