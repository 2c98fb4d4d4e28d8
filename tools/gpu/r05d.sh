#!/bin/bash
# round 5: the sched-barrier-wrapped operand fence: repeat probes, self-check builds, full GPU suite, C2 / C3
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05d; mkdir -p $O
timeout -k 10 200 python -u tools/dbg/field_repeat.py 200 > $O/field_repeat.txt 2>&1 || exit 1
timeout -k 10 300 python -u tools/dbg/selfcheck.py 20 > $O/selfcheck_default.txt 2>&1 || exit 2
for v in ws_check slots_check; do
  ACNERF_LIB=build_variants/libacnerf_$v.so timeout -k 10 300 python -u tools/dbg/selfcheck.py 10 > $O/selfcheck_$v.txt 2>&1 || exit 3
done
timeout -k 10 1200 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
timeout -k 10 200 python -u bench.py > $O/c2.json 2>$O/c2.err || exit 5
timeout -k 10 200 python -u bench.py --workload c3 > $O/c3.json 2>$O/c3.err || exit 6
