#!/bin/bash
# C5 on the final round-3 build: drop-in runtime_adapt line, rocprof kernel stats, PMC passes (HBM bytes, atomics)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03n
mkdir -p $O
timeout -k 10 400 python -u bench.py --workload c5 --driver runtime_adapt --no-cpu-baseline > $O/bench_c5ra.json 2> $O/bench_c5ra.err || { echo "c5ra failed"; tail -5 $O/bench_c5ra.err; exit 3; }
cut -c150-260 $O/bench_c5ra.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c5 -o run -- python3 bench.py --workload c5 --no-cpu-baseline > $O/prof_c5.log 2>&1 || { echo "prof failed"; exit 4; }
find $O/prof_c5 -type f ! -name '*kernel_stats.csv' -delete
i=0
for CTRS in "FETCH_SIZE" "WRITE_SIZE" "TCC_EA0_ATOMIC_sum TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 180 rocprofv3 --pmc $CTRS --output-format csv -d $O/pmc/p$i -o run -- python3 bench.py --workload c5 --no-graph --steps 4 --warmup 1 --no-cpu-baseline > $O/pmc_p$i.log 2>&1 || { echo "pass $i failed: $CTRS"; exit 5; }
done
python3 tools/pmc_summary_c5.py $O/pmc > $O/pmc_summary.txt
find $O/pmc -type f ! -name '*counter_collection.csv' -delete
cat $O/pmc_summary.txt | grep -E "adam|bwd_pairs"
