#!/bin/bash
# round-4 counters of the routed render (C3, C4 at S = 96) and the C2 render on the final build
set -o pipefail
export TMPDIR=/tmp
bash tools/pmc_r04.sh c3r --workload c3 --steps 20 --warmup 3 --no-cpu-baseline || exit 1
bash tools/pmc_r04.sh c4s96r --workload c4 --samples 96 --steps 2 --warmup 1 --no-cpu-baseline || exit 2
python tools/pmc_fold_r04.py gpurun_out/pmc_c3r render_routed_kernel 1048576 gpurun_out/r04_pmc_c3_routed.json r04 "render_routed_kernel (C3)"
python tools/pmc_fold_r04.py gpurun_out/pmc_c4s96r render_routed_kernel 61440000 gpurun_out/r04_pmc_c4s96_routed.json r04 "render_routed_kernel (C4, S = 96)"
