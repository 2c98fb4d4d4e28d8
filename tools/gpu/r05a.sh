#!/bin/bash
# round 5: self-check builds (with / without the operand fence), the full GPU suite, C2 / C3 bench lines
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05a; mkdir -p $O
for v in ws_check slots_check ws_check_nofence slots_check_nofence; do
  ACNERF_LIB=build_variants/libacnerf_$v.so timeout -k 10 300 python -u tools/dbg/selfcheck.py 10 > $O/selfcheck_$v.txt 2>&1 || exit 1
done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || exit 2
timeout -k 10 200 python -u bench.py > $O/c2.json 2>$O/c2.err || exit 3
timeout -k 10 200 python -u bench.py --workload c3 > $O/c3.json 2>$O/c3.err || exit 4
