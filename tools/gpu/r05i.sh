#!/bin/bash
# round 5: output-level run-to-run stress of candidate fence placements (default lib = fence + sched barriers)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05i; mkdir -p $O
timeout -k 10 400 python -u tools/dbg/selfcheck.py 60 > $O/st_default.txt 2>&1 || exit 1
for v in r04pad sbmem; do
  ACNERF_LIB=build_variants/libacnerf_$v.so timeout -k 10 400 python -u tools/dbg/selfcheck.py 60 > $O/st_$v.txt 2>&1 || exit 2
  ACNERF_LIB=build_variants/libacnerf_$v.so timeout -k 10 200 python -u tools/dbg/field_repeat.py 200 > $O/fr_$v.txt 2>&1 || exit 3
done
for v in sc2 sc2_r04pad sc2_sbmem; do
  ACNERF_LIB=build_variants/libacnerf_$v.so timeout -k 10 400 python -u tools/dbg/selfcheck.py 30 > $O/sc_$v.txt 2>&1 || exit 4
done
