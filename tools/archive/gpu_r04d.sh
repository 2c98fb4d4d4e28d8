#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
export ACNERF_LIB=$PWD/build_variants/libacnerf_rtdbg.so
RT_DEBUG=1 timeout -k 10 200 python -u tools/dbg/rt_det.py 2>&1 | grep -v -i 'warning\|amdgpu.ids'
