#!/bin/bash
# C5 Adam traffic: FETCH_SIZE / WRITE_SIZE / TCC hit-miss of adam_slots_kernel over the bench's own step sequence
# (eager, 5 + 30 steps, bitwise the graph replay), one rocprofv3 --pmc pass per set, each under its own limit
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04ai; mkdir -p $O
i=0
for CTRS in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum TCC_EA0_ATOMIC_sum"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $CTRS --output-format csv -d $O/p$i -o run -- python3 bench.py --workload c5 --no-graph --steps 30 --warmup 5 --no-cpu-baseline > $O/p$i.json 2> $O/p$i.err || { echo "pass $i failed: $CTRS"; tail -5 $O/p$i.err; exit 1; }
  find $O/p$i -type f ! -name '*counter_collection.csv' -delete
done
echo "pmc c5 done"
