#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03s
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_mlp_train_gpu.py tests/test_meta_gpu.py tests/test_train.py -m gpu -q \
  --timeout 240 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|ERROR" $O/pytest.log | head -20; tail -2 $O/pytest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
echo "== prefetch"; timeout -k 10 200 python -u tools/micro/mlp_bench.py 2>&1 | grep -v amdgpu.ids | tail -2 || exit 1
echo "== no prefetch"; ACNERF_LIB=build_variants/libacnerf_nopf.so timeout -k 10 200 python -u tools/micro/mlp_bench.py 2>&1 | grep -v amdgpu.ids | tail -2 || exit 1
