#!/bin/bash
# round 6: where do the slots self-check mismatches come from?  hash-feature self-check, one level in flight, no fence
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06b; mkdir -p $O
for v in sc2fc sc2d1 sc2nf sc2; do
  ACNERF_LIB=build_variants/libacnerf_$v.so timeout -k 10 300 python -u tools/dbg/selfcheck.py 10 > $O/sc_$v.txt 2>&1 || exit 2
done
