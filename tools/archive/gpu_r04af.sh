#!/bin/bash
# counters of the C4 (S = 256) render line, so every render line carries its measured traffic
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04af; mkdir -p $O
bash tools/pmc_r04.sh c4f --workload c4 --steps 2 --warmup 1 --no-cpu-baseline || exit 1
python tools/pmc_fold_r04.py gpurun_out/pmc_c4f render_slots_kernel 163840000 $O/r04_pmc_c4_slots.json r04 "render_slots_kernel (C4, S = 256)" > $O/fold_c4f.txt
cat $O/fold_c4f.txt
