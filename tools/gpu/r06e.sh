#!/bin/bash
# round 6: hash-feature self-check records (which evaluation is wrong, which levels)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06e; mkdir -p $O
for v in sc2fc fc; do
  ACNERF_LIB=build_variants/libacnerf_$v.so timeout -k 10 300 python -u tools/dbg/selfcheck.py 10 > $O/sc_$v.txt 2>&1 || exit 2
done
