#!/bin/bash
# hazard-pad determinism variants, the new GPU tests (batch independence, EP render / bounded exchange, AMP)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04o; mkdir -p $O
for v in; do
  export ACNERF_LIB=$PWD/build_variants/libacnerf_$v.so
  echo "== check $v"; timeout -k 10 150 python -u tools/dbg/rt_check.py 2>&1 | grep -v -i 'warning\|amdgpu.ids' || exit 1
done
unset ACNERF_LIB
timeout -k 10 400 python -u -m pytest tests/test_amp.py -m gpu -v -rP --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest_amp.log 2>&1
rc=$?; grep -E "passed|failed|FAILED|ERROR|AMPREPORT" $O/pytest_amp.log | tail -14
timeout -k 10 600 python -u -m pytest tests/test_batch_independence.py tests/test_expert_parallel.py -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc2=$?; grep -E "passed|failed|FAILED|ERROR" $O/pytest.log | tail -14; [ $rc -eq 0 ] && rc=$rc2
exit $rc
