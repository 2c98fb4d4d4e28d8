#!/bin/bash
# round 5: the early Adam pass on the side stream (ACN_ADAM_EARLY=2 beside the scatter, 3 after the marking forward): fixture tests, C5 A/B of mode 3
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05ai; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_train.py -k "early_adam_on_side_stream or forward_segment_marks or segment_maps or routed_adapt_step_matches" -q -m gpu -x --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for v in base early2 base2 early2b; do
  case $v in early*) export ACN_ADAM_EARLY=3;; *) export ACN_ADAM_EARLY=0;; esac
  timeout -k 10 240 python -u bench.py --workload c5 --steps 30 --warmup 5 --no-cpu-baseline > $O/c5_$v.json 2>$O/c5_$v.err || { tail -5 $O/c5_$v.err; exit 2; }
  python -c "import json;d=json.load(open('$O/c5_$v.json'));print('$v', d['ms_per_step'], d['roofline']['kernel_ms'])"
done
export ACN_ADAM_EARLY=3
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o run -- python3 bench.py --workload c5 --steps 4 --warmup 3 --no-cpu-baseline > $O/trace.log 2>&1 || exit 3
find $O/trace -type f ! -name '*kernel_trace.csv' -delete
