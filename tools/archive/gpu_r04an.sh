#!/bin/bash
# C2 on the work-shared render: counter passes (tools/pmc_r04.sh) folded into profiles/r04_pmc_c2_ws.json,
# then the default bench line (with the CPU baseline) and a rocprof kernel-stats run of the same command
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04an; mkdir -p $O
bash tools/pmc_r04.sh c2ws --steps 20 --no-cpu-baseline || exit 1
python tools/pmc_fold_r04.py gpurun_out/pmc_c2ws render_ws_kernel 1048576 $O/r04_pmc_c2_ws.json r04 "render_ws_kernel<1> (C2)" > $O/fold_c2ws.txt || exit 2
cat $O/fold_c2ws.txt | tail -5
cp $O/r04_pmc_c2_ws.json profiles/r04_pmc_c2_ws.json
timeout -k 10 300 python -u bench.py > $O/bench_c2.json 2> $O/bench_c2.err || { tail -3 $O/bench_c2.err; exit 3; }
python -c "import json; a=json.load(open('$O/bench_c2.json')); print('c2', a['value'], a['ms_per_step'], a['roofline']['kernel_ms'], a['roofline']['frac'], a['roofline']['traffic'], a['cpu_baseline']['value'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --no-cpu-baseline > $O/prof_c2.json 2>/dev/null || exit 4
f=$(find $O/prof -name '*kernel_stats.csv' | head -1); cp $f $O/c2_kernel_stats.csv
find $O/prof -type f ! -name '*kernel_stats.csv' -delete
grep -E "ray_order|render_" $O/c2_kernel_stats.csv | cut -c1-150
