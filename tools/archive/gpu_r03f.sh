#!/bin/bash
# split routed render: determinism per diagnostic variant
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03f
mkdir -p $O
timeout -k 10 120 python -u tools/dbg/split_dbg5.py 2>&1 | grep -v amdgpu.ids | tail -3 || exit 1
for v in gw t512; do
  ACNERF_LIB=build_variants/libacnerf_$v.so timeout -k 10 120 python -u tools/dbg/split_dbg5.py 2>&1 | grep -v amdgpu.ids | tail -3 || exit 1
done
timeout -k 10 600 python -u -m pytest tests/test_k8.py tests/test_gpu_kernels.py tests/test_expert_parallel.py tests/test_module_api.py tests/test_parallel.py -m gpu -q \
  --timeout 240 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1; echo "pytest rc=$?"; grep -E "FAILED|ERROR" $O/pytest.log | head -20; tail -2 $O/pytest.log
