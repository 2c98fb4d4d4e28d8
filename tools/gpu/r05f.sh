#!/bin/bash
# round 5: detailed slots self-check over three fence placements
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05f; mkdir -p $O
for v in slots_check2 slots_check2_r04pad slots_check2_nosb; do
  ACNERF_LIB=build_variants/libacnerf_$v.so timeout -k 10 300 python -u tools/dbg/selfcheck.py 10 > $O/sc_$v.txt 2>&1 || exit 1
done
