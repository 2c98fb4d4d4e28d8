#!/bin/bash
# routed vs slots render on one box: bench lines, C3 counters of both kernels, C4 expert layout, split recheck
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04s; mkdir -p $O
SL=$PWD/build_variants/libacnerf_slots.so
for w in "c3" "c4 --samples 96 --steps 5"; do
  t=${w%% *}
  timeout -k 10 200 python -u bench.py --workload $w --no-cpu-baseline > $O/${t}_routed.json 2>/dev/null || exit 3
  ACNERF_LIB=$SL timeout -k 10 200 python -u bench.py --workload $w --no-cpu-baseline > $O/${t}_slots.json 2>/dev/null || exit 4
  for v in split_exsel0 split_exsel1; do
    ACNERF_LIB=$PWD/build_variants/libacnerf_$v.so timeout -k 10 200 python -u bench.py --workload $w --no-cpu-baseline > $O/${t}_$v.json 2>/dev/null || exit 4
  done
  for v in routed slots split_exsel0 split_exsel1; do python -c "import json; a=json.load(open('$O/${t}_$v.json')); print('$t $v', a['value'], a['roofline']['kernel_ms'], a['ms_per_step'])"; done
done
timeout -k 10 300 python -u bench.py --workload c4 --samples 96 --steps 5 --layout expert --no-cpu-baseline > $O/c4s96_expert.json 2>$O/c4e.err || exit 5
python -c "import json; a=json.load(open('$O/c4s96_expert.json')); print('c4 expert', a['value'], a['ms_per_step'], a['roofline']['kernel_ms'])"
bash tools/pmc_r04.sh c3r --workload c3 --steps 20 --warmup 3 --no-cpu-baseline || exit 6
ACNERF_LIB=$SL bash tools/pmc_r04.sh c3s --workload c3 --steps 20 --warmup 3 --no-cpu-baseline || exit 7
python tools/pmc_fold_r04.py gpurun_out/pmc_c3r render_routed_kernel 1048576 $O/r04_pmc_c3_routed.json r04 "render_routed_kernel (C3)" > $O/fold_c3r.txt
python tools/pmc_fold_r04.py gpurun_out/pmc_c3s render_slots_kernel 1048576 $O/r04_pmc_c3_slots_same_box.json r04 "render_slots_kernel (C3)" > $O/fold_c3s.txt
cat $O/fold_c3r.txt $O/fold_c3s.txt
bash tools/gpu_r04r.sh
