#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
for v in accfirst pad; do
  export ACNERF_LIB=$PWD/build_variants/libacnerf_$v.so
  echo "== $v"
  timeout -k 10 200 python -u tools/dbg/rt_det2.py 2>&1 | grep -v -i 'warning\|amdgpu.ids'
done
