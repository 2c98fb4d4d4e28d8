#!/bin/bash
# C2 render per-wave timeline (diagnostic build -DACN_DIAG_WAVETIME=1)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
ACNERF_LIB=build_variants/libacnerf_wavetime.so timeout -k 10 200 python -u tools/micro/wave_times.py > gpurun_out/wave_times.log 2>&1; rc=$?
cat gpurun_out/wave_times.log | grep -v amdgpu.ids; exit $rc
