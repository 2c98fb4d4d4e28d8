#!/bin/bash
# final-build check: the whole -m gpu suite and smoke()
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04w; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_all.log 2>&1
rc=$?; tail -15 $O/pytest_all.log | grep -E "passed|failed|FAILED|ERROR"; echo "suite rc=$rc"
[ $rc -le 1 ] || exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke OK')" 2>&1 | tail -2
exit $rc
