#!/bin/bash
# round 3: whole GPU suite + smoke + the training-parity spread table
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03j
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?
grep -E "FAILED|ERROR" $O/pytest.log | head -30
tail -2 $O/pytest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1; echo "smoke rc=$?"; tail -2 $O/smoke.log
timeout -k 10 400 python -u tools/train_spread.py --out $O/train_spread.json > $O/train_spread.log 2>&1; echo "spread rc=$?"; tail -5 $O/train_spread.log
