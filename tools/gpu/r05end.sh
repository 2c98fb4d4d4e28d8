#!/bin/bash
# round 5, last check of the committed tree: full GPU suite and smoke
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05end; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/suite.log 2>&1; rc=$?
tail -1 $O/suite.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/suite.log | head; exit 1; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 2
tail -1 $O/smoke.log
