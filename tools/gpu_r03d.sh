#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03d
mkdir -p $O
timeout -k 10 150 python -u tools/dbg/split_dbg3.py > $O/dbg3.log 2>&1; echo "dbg3 rc=$?"; grep -v amdgpu.ids $O/dbg3.log | tail -8
for v in nofold lockstep; do echo "== $v"; ACNERF_LIB=build_variants/libacnerf_$v.so timeout -k 10 150 python -u tools/dbg/split_dbg2.py 2>&1 | grep -v amdgpu.ids | head -8 || exit 1; done
timeout -k 10 400 python -u tools/train_spread.py --out $O/train_spread.json > $O/train_spread.log 2>&1; echo "spread rc=$?"; tail -5 $O/train_spread.log
timeout -k 10 600 python -u -m pytest tests/test_train.py -k "deterministic or drop_in or ragged" tests/test_meta_gpu.py tests/test_expert_parallel.py -m gpu -v \
  --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
echo "pytest rc=$?"; grep -E "FAILED|ERROR" $O/pytest.log | head -20; tail -2 $O/pytest.log
