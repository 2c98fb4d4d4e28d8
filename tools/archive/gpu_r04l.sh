#!/bin/bash
# hazard-pad variants (determinism self-check + C2/C3 rate), new GPU tests, float64 spread
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04l; mkdir -p $O
for v in nop1 nop3; do
  export ACNERF_LIB=$PWD/build_variants/libacnerf_$v.so
  echo "== check $v"; timeout -k 10 200 python -u tools/dbg/rt_check.py 2>&1 | grep -v -i 'warning\|amdgpu.ids' || exit 1
done
unset ACNERF_LIB
timeout -k 10 900 python -u -m pytest tests/test_batch_independence.py tests/test_expert_parallel.py tests/test_k8.py tests/test_gpu_kernels.py -m gpu -v --timeout 600 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; grep -E "passed|failed|FAILED|ERROR" $O/pytest.log | tail -12
timeout -k 10 900 python -u -m pytest tests/test_train.py tests/test_meta_gpu.py -m gpu -k "alternating or drop_in or ragged or state_dict or graphed or segment" -v --timeout 600 --timeout-method thread -p no:cacheprovider > $O/pytest2.log 2>&1
rc2=$?; grep -E "passed|failed|FAILED|ERROR" $O/pytest2.log | tail -12; [ $rc -eq 0 ] && rc=$rc2
for v in base perf_nop0 perf_nop1; do
  if [ $v = base ]; then unset ACNERF_LIB; else export ACNERF_LIB=$PWD/build_variants/libacnerf_$v.so; fi
  timeout -k 10 200 python -u bench.py --no-cpu-baseline > $O/c2_$v.json 2>/dev/null || exit 3
  timeout -k 10 200 python -u bench.py --workload c3 --steps 100 --no-cpu-baseline > $O/c3_$v.json 2>/dev/null || exit 4
  python -c "import json; a=json.load(open('$O/c2_$v.json')); b=json.load(open('$O/c3_$v.json')); print('$v', 'c2', a['value'], a['roofline']['kernel_ms'], 'c3', b['value'], b['roofline']['kernel_ms'])"
done
unset ACNERF_LIB
timeout -k 10 200 python -u bench.py --workload c4 --samples 96 --steps 3 --no-cpu-baseline > $O/c4s96.json 2>/dev/null || exit 5
python -c "import json; a=json.load(open('$O/c4s96.json')); print('c4s96', a['value'], a['roofline']['kernel_ms'])"
timeout -k 10 400 python -u tools/train_f64_spread.py --out $O/train_f64_spread.json 2>&1 | grep -v -i 'warning\|amdgpu.ids' | tail -30
exit $rc
