#!/bin/bash
# round 5: bisect the field kernel's run-to-run differences over fence variants
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05c; mkdir -p $O
timeout -k 10 200 python -u tools/dbg/field_repeat.py 100 > $O/fr_default.txt 2>&1 || exit 1
for v in v_nofence v_mem v_sb v_r04pad r04; do
  ACNERF_LIB=build_variants/libacnerf_$v.so timeout -k 10 200 python -u tools/dbg/field_repeat.py 100 > $O/fr_$v.txt 2>&1 || exit 2
done
