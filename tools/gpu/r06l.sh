#!/bin/bash
# round 6: with buffer-load gathers, is the operand fence still needed?  field-kernel repeats and slots self-check
# with and without it; the training MLP without it (determinism test + meta step)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06l; mkdir -p $O
unset ACNERF_LIB
timeout -k 10 300 python -u tools/dbg/field_repeat.py 200 > $O/fr_default.txt 2>&1 || exit 1
ACNERF_LIB=build_variants/libacnerf_nf.so timeout -k 10 300 python -u tools/dbg/field_repeat.py 200 > $O/fr_nf.txt 2>&1 || exit 1
ACNERF_LIB=build_variants/libacnerf_sc2.so timeout -k 10 300 python -u tools/dbg/selfcheck.py 30 > $O/sc_sc2.txt 2>&1 || exit 2
ACNERF_LIB=build_variants/libacnerf_sc2nf.so timeout -k 10 300 python -u tools/dbg/selfcheck.py 30 > $O/sc_sc2nf.txt 2>&1 || exit 2
ACNERF_LIB=build_variants/libacnerf_mlpnf.so timeout -k 10 400 python -u -m pytest -x -q --timeout 300 tests/test_determinism_gpu.py > $O/det_mlpnf.txt 2>&1 || exit 3
for rep in 1 2; do
  unset ACNERF_LIB
  timeout -k 10 300 python -u bench.py --workload meta --no-cpu-baseline > $O/meta_default_$rep.json 2> $O/meta_default_$rep.err || exit 4
  ACNERF_LIB=build_variants/libacnerf_mlpnf.so timeout -k 10 300 python -u bench.py --workload meta --no-cpu-baseline > $O/meta_mlpnf_$rep.json 2> $O/meta_mlpnf_$rep.err || exit 4
done
