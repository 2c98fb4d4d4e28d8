#!/bin/bash
# round 6: counter passes of the final render build (C2 render_ws_kernel, C3 / C4-S96 render_slots_kernel)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06p; mkdir -p $O
timeout -k 10 500 bash tools/pmc_r04.sh r06_c2 --workload c2 --steps 20 --no-cpu-baseline > $O/pmc_c2.log 2>&1 || exit 1
timeout -k 10 500 bash tools/pmc_r04.sh r06_c3 --workload c3 --steps 20 --no-cpu-baseline > $O/pmc_c3.log 2>&1 || exit 2
timeout -k 10 500 bash tools/pmc_r04.sh r06_c4s96 --workload c4 --samples 96 --steps 3 --warmup 1 --no-cpu-baseline > $O/pmc_c4s96.log 2>&1 || exit 3
