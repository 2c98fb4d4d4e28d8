#!/bin/bash
# ray_order_kernel with one coordinate pass: order / render tests, then C2 kernel stats and the bench line
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04az; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_batch_independence.py tests/test_render_ws.py tests/test_gpu_kernels.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 50 --no-cpu-baseline > $O/c2_prof.json 2>/dev/null || exit 2
f=$(find $O/prof -name '*kernel_stats.csv' | head -1); cp $f $O/c2_kernel_stats.csv
find $O/prof -type f ! -name '*kernel_stats.csv' -delete
grep -E "ray_order|render_ws" $O/c2_kernel_stats.csv | cut -c1-150
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --no-cpu-baseline > $O/c2_$i.json 2>/dev/null || exit 3
  python -c "import json; a=json.load(open('$O/c2_$i.json')); print('c2', a['value'], a['ms_per_step'], a['roofline']['kernel_ms'])"
done
