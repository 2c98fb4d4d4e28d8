#!/bin/bash
# final round-3 build (slots render folds the SH bias on every path): whole GPU suite + smoke, C2 / C3 / C4-S96 / meta bench lines, meta rocprof
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03ac
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?
grep -E "FAILED|ERROR" $O/pytest.log | head -30
tail -2 $O/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -5 $O/smoke.log; exit 2; }
tail -1 $O/smoke.log
timeout -k 10 400 python -u bench.py --steps 20 > $O/bench_c2.json 2> $O/bench_c2.err || { echo "bench failed"; tail -5 $O/bench_c2.err; exit 3; }
cut -c1-200 $O/bench_c2.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_meta -o run -- python3 bench.py --workload meta --steps 3 --warmup 1 --no-cpu-baseline > $O/prof_meta.log 2>&1 || { echo "prof meta failed"; exit 4; }
find $O/prof_meta -type f ! -name '*kernel_stats.csv' -delete
timeout -k 10 400 python -u bench.py --workload meta > $O/bench_meta.json 2> $O/bench_meta.err || { echo "meta failed"; exit 5; }
cut -c1-200 $O/bench_meta.json
timeout -k 10 300 python -u bench.py --workload c3 --steps 50 --no-cpu-baseline > $O/bench_c3.json 2> $O/bench_c3.err || { echo "c3 failed"; exit 6; }
cut -c1-200 $O/bench_c3.json
timeout -k 10 300 python -u bench.py --workload c4 --samples 96 --steps 3 --no-cpu-baseline > $O/bench_c4s96.json 2> $O/bench_c4s96.err || { echo "c4 failed"; exit 7; }
cut -c1-200 $O/bench_c4s96.json
echo "r03ac done"
