#!/bin/bash
# round 3: drop-in runtime_adapt / train_step through the graphed steps (SlottedAdam), their tests and bench lines
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03b
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_train.py tests/test_meta_gpu.py tests/test_graph_gpu.py tests/test_loss_gpu.py tests/test_expert_parallel.py -m gpu -x -v \
  --timeout 240 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { echo "pytest failed"; grep -E "FAIL|Error|error" $O/pytest.log | head -30; tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 300 python -u bench.py --workload c5 --no-cpu-baseline > $O/bench_c5.json 2> $O/bench_c5.err || { echo "bench c5 failed"; tail $O/bench_c5.err; exit 3; }
cat $O/bench_c5.json
timeout -k 10 300 python -u bench.py --workload c5 --driver runtime_adapt --no-cpu-baseline > $O/bench_c5_ra.json 2> $O/bench_c5_ra.err || { echo "bench c5 ra failed"; tail $O/bench_c5_ra.err; exit 4; }
cat $O/bench_c5_ra.json
timeout -k 10 300 python -u bench.py --workload meta --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_meta.json 2> $O/bench_meta.err || { echo "bench meta failed"; tail $O/bench_meta.err; exit 5; }
cat $O/bench_meta.json
echo "r03b done"
