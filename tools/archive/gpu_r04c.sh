#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04c; mkdir -p $O
for v in base exsel slots; do
  if [ $v = base ]; then unset ACNERF_LIB; else export ACNERF_LIB=$PWD/build_variants/libacnerf_$v.so; fi
  echo "== $v"
  timeout -k 10 200 python -u tools/dbg/rt_det.py 2>&1 | grep -v Warning || exit 1
done
