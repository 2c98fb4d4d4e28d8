#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
for v in dbg2 static sync depth1; do
  export ACNERF_LIB=$PWD/build_variants/libacnerf_$v.so
  VARIANT=$v timeout -k 10 200 python -u tools/dbg/rt_det4.py 2>&1 | grep -v -i 'warning\|amdgpu.ids'
done
