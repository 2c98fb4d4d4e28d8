#!/bin/bash
# round-3 checkpoint: whole GPU suite + smoke, the default bench line (C2, CPU baseline), rocprof of C2
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03r
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?
grep -E "FAILED|ERROR" $O/pytest.log | head -30
tail -2 $O/pytest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1; echo "smoke rc=$?"; tail -1 $O/smoke.log
timeout -k 10 400 python -u bench.py --steps 20 > $O/bench_c2.json 2> $O/bench_c2.err || { echo "bench failed"; tail -5 $O/bench_c2.err; exit 3; }
cut -c1-300 $O/bench_c2.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c2 -o run -- python3 bench.py --steps 20 --no-cpu-baseline > $O/prof_c2.log 2>&1 || { echo "prof failed"; exit 4; }
find $O/prof_c2 -type f ! -name '*kernel_stats.csv' -delete
echo "r03r done"
