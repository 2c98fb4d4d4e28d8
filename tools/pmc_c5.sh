#!/bin/bash
# PMC passes over the C5 routed step (eager RoutedAdaptStep: the same kernels as the graph replay),
# one rocprofv3 --pmc run per counter set, each under its own hard limit.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/pmc_c5
mkdir -p $OUT
i=0
for CTRS in "FETCH_SIZE" "WRITE_SIZE" "TCC_EA0_ATOMIC_sum TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 180 rocprofv3 --pmc $CTRS --output-format csv -d $OUT/p$i -o run -- python3 bench.py --workload c5 --no-graph --steps 4 --warmup 1 --no-cpu-baseline > $OUT/p$i.log 2>&1 || { echo "pass $i failed: $CTRS"; exit 1; }
done
echo "pmc c5 done"
