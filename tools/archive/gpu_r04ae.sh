#!/bin/bash
# consumer-side fp16x3 dW (variant dwcsplit): role timings, MLP / training / meta parity, meta A/B
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04ae; mkdir -p $O
V=$PWD/build_variants/libacnerf_dwcsplit.so
for v in base dwcsplit; do
  if [ $v = base ]; then unset ACNERF_LIB; else export ACNERF_LIB=$V; fi
  timeout -k 10 120 python -u tools/micro/mlp_bwd_roles.py $v 2>&1 | grep "fp16x3" || exit 1
done
ACNERF_LIB=$V timeout -k 10 700 python -u -m pytest tests/test_mlp_train_gpu.py tests/test_train.py tests/test_meta_gpu.py -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_v.log 2>&1
rc=$?; tail -3 $O/pytest_v.log; grep FAILED $O/pytest_v.log | head; [ $rc -le 1 ] || exit $rc
for v in base dwcsplit base dwcsplit; do
  if [ $v = base ]; then unset ACNERF_LIB; else export ACNERF_LIB=$V; fi
  timeout -k 10 300 python -u bench.py --workload meta --no-cpu-baseline > $O/meta_$v.json 2>$O/meta_$v.err || exit 3
  python -c "import json; a=json.load(open('$O/meta_$v.json')); r=a['roofline']; print('meta $v', a['value'], a['ms_per_step'], r.get('kernel_ms'))"
done
exit $rc
