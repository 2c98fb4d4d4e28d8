#!/bin/bash
# routed step with the background backward on a side stream (ACN_BG_SIDE) + copy-free jitter / loss: training
# suites, then the C5 A/B against the head's backward in line (ACN_BG_SIDE=0), alternating
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04aw; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_train.py tests/test_amp.py tests/test_graph_keepalive.py tests/test_expert_parallel.py -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; grep -E "passed|failed|FAILED" $O/pytest.log | tail -6; echo "tests rc=$rc"; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for b in 1 0; do
    ACN_BG_SIDE=$b timeout -k 10 200 python -u bench.py --workload c5 --no-cpu-baseline > $O/c5_bg${b}_$i.json 2>$O/c5_bg${b}_$i.err || { tail -3 $O/c5_bg${b}_$i.err; exit 3; }
    python -c "import json; a=json.load(open('$O/c5_bg${b}_$i.json')); r=a['roofline']; print('c5 bg_side=$b', a['value'], a['ms_per_step'], r['kernel_ms'], r['secondary'].get('kernel_ms'), a['val_psnr_db'])"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --workload c5 --no-cpu-baseline > $O/c5_prof.json 2>/dev/null || exit 4
f=$(find $O/prof -name '*kernel_stats.csv' | head -1); cp $f $O/c5_kernel_stats.csv
find $O/prof -type f ! -name '*kernel_stats.csv' -delete
grep -E "routed_scan|background_bwd|bg_bwd_reduce|adam_slots|hashgrid_bwd" $O/c5_kernel_stats.csv | cut -c1-120
