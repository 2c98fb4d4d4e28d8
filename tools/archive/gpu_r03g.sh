#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 120 python -u tools/dbg/split_dbg5.py 2>&1 | grep -v amdgpu.ids | tail -2 || exit 1
ACNERF_LIB=build_variants/libacnerf_exsel.so timeout -k 10 120 python -u tools/dbg/split_dbg5.py 2>&1 | grep -v amdgpu.ids | tail -2 || exit 1
