#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 200 python -u tools/dbg/field_perm.py 2>&1 | grep -v -i 'warning\|amdgpu.ids' || exit 1
export ACNERF_LIB=$PWD/build_variants/libacnerf_r1.so
echo "== R=1"
timeout -k 10 200 python -u tools/dbg/rt_det.py 2>&1 | grep -v -i 'warning\|amdgpu.ids'
