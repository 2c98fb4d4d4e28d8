#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
export ACNERF_LIB=$PWD/build_variants/libacnerf_checknop.so
timeout -k 10 200 python -u tools/dbg/rt_check.py 2>&1 | grep -v -i 'warning\|amdgpu.ids'
unset ACNERF_LIB
timeout -k 10 400 python -u tools/train_f64_spread.py --out gpurun_out/train_f64_spread.json 2>&1 | grep -v -i 'warning\|amdgpu.ids' | tail -40
