#!/bin/bash
# round 6: hash-feature mismatch rate under candidate fixes (sensitive self-check layout), and the production layout
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06g; mkdir -p $O
for v in sc2fc fcd1 fcx2; do
  ACNERF_LIB=build_variants/libacnerf_$v.so timeout -k 10 300 python -u tools/dbg/selfcheck.py 20 > $O/sc_$v.txt 2>&1 || exit 2
done
ACNERF_LIB=build_variants/libacnerf_fc.so timeout -k 10 300 python -u tools/dbg/selfcheck.py 40 > $O/sc_fc.txt 2>&1 || exit 3
