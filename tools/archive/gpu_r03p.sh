#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
for lib in "" build_variants/libacnerf_s768.so; do
  ACNERF_LIB=${lib:-adaptive_city_nerf_amd/libacnerf.so} timeout -k 10 300 python -u bench.py --workload c3 --no-cpu-baseline 2>/dev/null | cut -c150-230 || exit 1
  ACNERF_LIB=${lib:-adaptive_city_nerf_amd/libacnerf.so} timeout -k 10 300 python -u bench.py --workload c4 --samples 96 --no-cpu-baseline 2>/dev/null | cut -c150-230 || exit 1
done
