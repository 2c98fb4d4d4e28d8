#!/bin/bash
# round 5: C3 with the multi-expert rays visited after the single-expert ones (render_slots_kernel rounds of
# uniform cost) against the default plan
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05z; mkdir -p $O
for v in default multi default2 multi2; do
  case $v in multi*) X=--diag-multi-last;; *) X=;; esac
  timeout -k 10 200 python -u bench.py --workload c3 --no-cpu-baseline $X > $O/c3_$v.json 2>$O/c3_$v.err || { tail -5 $O/c3_$v.err; exit 1; }
  python -c "import json;d=json.load(open('$O/c3_$v.json'));print('c3 $v', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['config'].get('plan'))"
done
