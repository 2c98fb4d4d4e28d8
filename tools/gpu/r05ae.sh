#!/bin/bash
# round 5: C5 with the background head's backward on the side stream (beside the MLP backward), A/B; and an
# eager-step kernel trace (are the ~6 us gaps before the table scatter / clip / bump graph-only?)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05ae; mkdir -p $O
for v in base side base2 side2; do
  case $v in side*) export ACN_BG_SIDE=1;; *) export ACN_BG_SIDE=0;; esac
  timeout -k 10 240 python -u bench.py --workload c5 --steps 30 --warmup 5 --no-cpu-baseline > $O/c5_$v.json 2>$O/c5_$v.err || exit 1
  python -c "import json;d=json.load(open('$O/c5_$v.json'));print('$v', d['ms_per_step'], d['roofline']['kernel_ms'])"
done
export ACN_BG_SIDE=0
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/eager -o run -- python3 bench.py --workload c5 --steps 4 --warmup 3 --no-graph --no-cpu-baseline > $O/eager.log 2>&1 || exit 2
find $O/eager -type f ! -name '*kernel_trace.csv' -delete
export ACN_BG_SIDE=1
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/side -o run -- python3 bench.py --workload c5 --steps 4 --warmup 3 --no-cpu-baseline > $O/side.log 2>&1 || exit 3
find $O/side -type f ! -name '*kernel_trace.csv' -delete
