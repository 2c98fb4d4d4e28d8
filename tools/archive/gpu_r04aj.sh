#!/bin/bash
# adam_slots_kernel occupancy A/B on C5: base (4 vectors/lane, 166 VGPRs, 3 waves/SIMD), u2 (2 vectors, 94 VGPRs,
# 5 waves/SIMD), u2w6 (2 vectors, 6 waves/SIMD), u2pipe (u2 + map bytes one iteration ahead), w4 (4 vectors forced
# to 4 waves/SIMD, 10 VGPRs spilled); alternating runs on one box
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04aj; mkdir -p $O
bash tools/ab_c5.sh $O/ab_c5.txt base u2 u2w6 u2pipe w4 base u2 u2w6 u2pipe w4 || exit 2
