#!/bin/bash
# round 3 re-entry: state of the whole GPU suite (no -x) + the split routed render's ray-list diagnostic
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03e
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?
grep -E "FAILED|ERROR" $O/pytest.log | head -40
tail -3 $O/pytest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 150 python -u tools/dbg/split_dbg4.py > $O/dbg4.log 2>&1; echo "dbg4 rc=$?"; grep -v amdgpu.ids $O/dbg4.log | tail -8
