#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
export ACNERF_LIB=$PWD/build_variants/libacnerf_dbg2.so
timeout -k 10 200 python -u tools/dbg/rt_det3.py 2>&1 | grep -v -i 'warning\|amdgpu.ids'
