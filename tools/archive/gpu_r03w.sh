#!/bin/bash
# rocprof kernel stats of the meta / C5 / C3 lines on the current build (+ their bench lines)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03w
mkdir -p $O
for spec in "meta:--workload meta --steps 3 --warmup 1" "c5:--workload c5" "c3:--workload c3 --steps 50"; do
  t=${spec%%:*}; args=${spec#*:}
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$t -o run -- python3 bench.py $args --no-cpu-baseline > $O/prof_$t.log 2>&1 || { echo "prof $t failed"; exit 4; }
  find $O/prof_$t -type f ! -name '*kernel_stats.csv' -delete
done
timeout -k 10 400 python -u bench.py --workload c5 > $O/bench_c5.json 2> $O/bench_c5.err || { echo "c5 failed"; exit 3; }
cut -c150-260 $O/bench_c5.json
echo "r03w done"
