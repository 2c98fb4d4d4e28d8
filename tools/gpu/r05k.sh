#!/bin/bash
# round 5: is it a wait-count (memory ordering) problem?  The flaky builds with every s_waitcnt forced to zero
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05k; mkdir -p $O
for v in nosb nosb_fz; do
  ACNERF_LIB=build_variants/libacnerf_$v.so timeout -k 10 300 python -u tools/dbg/field_repeat.py 100 > $O/fr_$v.txt 2>&1 || exit 1
done
for v in sc2 sc2_fz; do
  ACNERF_LIB=build_variants/libacnerf_$v.so timeout -k 10 400 python -u tools/dbg/selfcheck.py 30 > $O/sc_$v.txt 2>&1 || exit 2
done
