#!/bin/bash
# compacted clip-norm plan + background-gradient reduction: the training suites, C5 rocprof + bench line
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03z
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_train.py tests/test_graph_gpu.py tests/test_meta_gpu.py tests/test_expert_parallel.py tests/test_loss_gpu.py -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?
grep -E "FAILED|ERROR" $O/pytest.log | head -30
tail -2 $O/pytest.log
[ $rc -eq 0 ] || [ $rc -eq 4 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c5 -o run -- python3 bench.py --workload c5 --no-cpu-baseline > $O/prof_c5.log 2>&1 || { echo "prof c5 failed"; exit 4; }
find $O/prof_c5 -type f ! -name '*kernel_stats.csv' -delete
timeout -k 10 400 python -u bench.py --workload c5 --no-cpu-baseline > $O/bench_c5.json 2> $O/bench_c5.err || { echo "c5 failed"; exit 5; }
cut -c1-260 $O/bench_c5.json
echo "r03z done"
