#!/bin/bash
# round 5: the fused C5 glue (composite + MSE + backward in one launch, norm + clip in one launch): bitwise test
# against the separate launches, the routed-step suites, then C5 A/B on one box and a kernel trace
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05s; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_routed_glue.py tests/test_train.py tests/test_amp.py -q -m gpu -x --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
for tag in fused plain fused2 plain2; do
  case $tag in plain*) export ACN_FUSED_COMPOSITE=0 ACN_FUSED_CLIP=0;; *) export ACN_FUSED_COMPOSITE=1 ACN_FUSED_CLIP=1;; esac
  timeout -k 10 240 python -u bench.py --workload c5 --steps 30 --warmup 5 --no-cpu-baseline > $O/c5_$tag.json 2>$O/c5_$tag.err || exit 2
  python -c "import json;d=json.load(open('$O/c5_$tag.json'));print('$tag', d['ms_per_step'], d['roofline']['kernel_ms'])"
done
export ACN_FUSED_COMPOSITE=1 ACN_FUSED_CLIP=1
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/c5trace -o run -- python3 bench.py --workload c5 --steps 4 --warmup 3 --no-cpu-baseline > $O/c5trace.log 2>&1 || exit 3
find $O/c5trace -type f ! -name '*kernel_trace.csv' -delete
