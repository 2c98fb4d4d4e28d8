#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
ACNERF_LIB=build_variants/libacnerf_dwdiag.so timeout -k 10 120 python -u tools/micro/mlp_dw_diag.py 2>&1 | grep -v amdgpu.ids | tail -12
