#!/bin/bash
# meta step with each task's rays in direction-cell order (--meta-task-order 1) vs as drawn: meta GPU tests
# with the order on, then the A/B (fp32-accurate and use_amp), alternating
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04au; mkdir -p $O
ACN_META_TASK_ORDER=1 timeout -k 10 600 python -u -m pytest tests/test_meta_gpu.py tests/test_amp.py -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; grep -E "passed|failed|FAILED" $O/pytest.log | tail -6; echo "tests rc=$rc"
for i in 1 2; do
  for o in 0 1; do
    for m in fp16x3 amp; do
      timeout -k 10 300 python -u bench.py --workload meta --mlp-precision $m --meta-task-order $o --no-cpu-baseline > $O/meta_${m}_o${o}_$i.json 2>$O/meta_${m}_o${o}_$i.err || { tail -3 $O/meta_${m}_o${o}_$i.err; exit 3; }
      python -c "import json; a=json.loads(open('$O/meta_${m}_o${o}_$i.json').read().strip().splitlines()[-1]); print('meta $m order=$o', a['value'], a['ms_per_step'], a.get('loss'))"
    done
  done
done
