#!/bin/bash
# round 6, final build: counter passes of the render workloads (C2, C3, C4-S96) for the bench lines' traffic
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06v; mkdir -p $O
timeout -k 10 600 bash tools/pmc_r04.sh r06v_c2 --workload c2 --no-cpu-baseline > $O/pmc_c2.log 2>&1 || exit 1
timeout -k 10 600 bash tools/pmc_r04.sh r06v_c3 --workload c3 --no-cpu-baseline > $O/pmc_c3.log 2>&1 || exit 2
timeout -k 10 900 bash tools/pmc_r04.sh r06v_c4s96 --workload c4 --samples 96 --steps 3 --no-cpu-baseline > $O/pmc_c4s96.log 2>&1 || exit 3
