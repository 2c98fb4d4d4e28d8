#!/bin/bash
# Diagnostic: is C3's per-sample deficit vs C2 the experts' finer hash-grid cells?  C3 and C4 S=96 with every
# expert given the whole-scene box (C2's cell size), plus L2 hit/miss counters for those runs.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04ag; mkdir -p $O
run() { # tag args...
  local t=$1; shift
  timeout -k 10 200 python -u bench.py --no-cpu-baseline "$@" > $O/$t.json 2>$O/$t.err || { tail -5 $O/$t.err; exit 3; }
  python -c "import json; a=json.load(open('$O/$t.json')); print('$t', a['value'], a['ms_per_step'], a['roofline'].get('kernel_ms'))"
}
run c2
run c3 --workload c3
run c3_gbox --workload c3 --diag-expert-box global
run c3_gbox_shared --workload c3 --diag-expert-box global --diag-shared-table
run c4s96 --workload c4 --samples 96
run c4s96_gbox --workload c4 --samples 96 --diag-expert-box global
for t in "c3:--workload c3" "c3_gbox:--workload c3 --diag-expert-box global" "c2:" "c4s96_gbox:--workload c4 --samples 96 --diag-expert-box global"; do
  tag=${t%%:*}; args=${t#*:}
  timeout -s KILL 180 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $O/pmc_$tag -o run -- python3 bench.py --no-cpu-baseline --steps 10 $args \
      > $O/pmc_$tag.log 2>&1 || { echo "pmc $tag failed"; tail -5 $O/pmc_$tag.log; exit 4; }
  find $O/pmc_$tag -type f ! -name '*counter_collection.csv' -delete
done
echo done
