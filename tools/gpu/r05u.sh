#!/bin/bash
# round 5 final build: the full GPU suite and smoke
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05u; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/suite.log 2>&1; rc=$?
tail -3 $O/suite.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 2
tail -2 $O/smoke.log
