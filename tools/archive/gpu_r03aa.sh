#!/bin/bash
# inner-loop background cache: meta / graph / train suites, meta rocprof + bench line
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03aa
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_meta_gpu.py tests/test_graph_gpu.py tests/test_train.py -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?
grep -E "FAILED|ERROR" $O/pytest.log | head -30
tail -2 $O/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_meta -o run -- python3 bench.py --workload meta --steps 3 --warmup 1 --no-cpu-baseline > $O/prof_meta.log 2>&1 || { echo "prof meta failed"; exit 4; }
find $O/prof_meta -type f ! -name '*kernel_stats.csv' -delete
timeout -k 10 400 python -u bench.py --workload meta > $O/bench_meta.json 2> $O/bench_meta.err || { echo "meta failed"; exit 5; }
cut -c1-200 $O/bench_meta.json
echo "r03aa done"
