#!/bin/bash
# the fp16x3 weight-gradient stage in the producer / consumer MLP backward (variant dwf16x3): parity, then A/B
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04v; mkdir -p $O
V=$PWD/build_variants/libacnerf_dwf16x3.so
ACNERF_LIB=$V timeout -k 10 600 python -u -m pytest tests/test_mlp_train_gpu.py tests/test_train.py tests/test_meta_gpu.py -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_v.log 2>&1
rc=$?; tail -4 $O/pytest_v.log; echo "variant tests rc=$rc"
[ $rc -le 1 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_meta_gpu.py -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "state_dict or graphed" > $O/pytest_base.log 2>&1
echo "base meta tests rc=$? $(tail -1 $O/pytest_base.log)"
for v in base dwf16x3 base dwf16x3; do
  if [ $v = base ]; then unset ACNERF_LIB; else export ACNERF_LIB=$V; fi
  timeout -k 10 300 python -u bench.py --workload meta --no-cpu-baseline > $O/meta_$v.json 2>$O/meta_$v.err || exit 3
  python -c "import json; a=json.load(open('$O/meta_$v.json')); r=a['roofline']; print('meta $v', a['value'], a['ms_per_step'], r.get('kernel_ms'), r.get('frac'))"
done

for v in base band1 base band1; do
  if [ $v = base ]; then unset ACNERF_LIB; else export ACNERF_LIB=$PWD/build_variants/libacnerf_$v.so; fi
  timeout -k 10 200 python -u bench.py --workload c3 --no-cpu-baseline > $O/c3_$v.json 2>/dev/null || exit 4
  python -c "import json; a=json.load(open('$O/c3_$v.json')); print('c3 $v', a['value'], a['roofline']['kernel_ms'])"
done
exit $rc
