#!/bin/bash
# direction-cell visiting order in the differentiable training render: training / meta suites, then meta A/B
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04ac; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_meta_gpu.py tests/test_train.py tests/test_amp.py tests/test_module_api.py tests/test_occ_gpu.py -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; grep -E "FAILED" $O/pytest.log | head; [ $rc -le 1 ] || exit $rc
for o in 1 0 1 0; do
  ACN_TRAIN_ORDER=$o timeout -k 10 300 python -u bench.py --workload meta --no-cpu-baseline > $O/meta_o$o.json 2>$O/meta_o$o.err || exit 3
  python -c "import json; a=json.load(open('$O/meta_o$o.json')); r=a['roofline']; print('meta order=$o', a['value'], a['ms_per_step'], r.get('kernel_ms'))"
done
exit $rc
