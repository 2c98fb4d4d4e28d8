#!/bin/bash
# round 3 bench refresh: C2 / C5 (with CPU baselines), C5 through the drop-in runtime_adapt, meta, C3 / C4 / C4-S96,
# and rocprof kernel stats of C2 (the driver's 20 steps), C5 and meta.  Each step under its own limit.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03k
mkdir -p $O
keep_stats() { find "$1" -type f ! -name '*kernel_stats.csv' -delete; }
b() { n=$1; shift; timeout -k 10 300 python -u bench.py "$@" > $O/bench_$n.json 2> $O/bench_$n.err || { echo "bench $n failed"; tail -5 $O/bench_$n.err; exit 3; }; echo "$n: $(cut -c1-220 $O/bench_$n.json)"; }
b c2 --steps 20
b c5
b c5ra --workload c5 --driver runtime_adapt --no-cpu-baseline
b meta --workload meta --steps 10 --warmup 2 --no-cpu-baseline
b c3 --workload c3 --no-cpu-baseline
b c4 --workload c4 --no-cpu-baseline
b c4s96 --workload c4 --samples 96 --no-cpu-baseline
for spec in "c2:--steps 20" "c5:--workload c5" "meta:--workload meta --steps 3 --warmup 1"; do
  t=${spec%%:*}; args=${spec#*:}
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$t -o run -- python3 bench.py $args --no-cpu-baseline > $O/prof_$t.log 2>&1 || { echo "prof $t failed"; exit 4; }
  keep_stats $O/prof_$t
done
echo "r03k done"
