#!/bin/bash
# work-shared single-expert render (render_ws_kernel): bitwise test against render_kernel + the render suites,
# then C2 (rocprof stats + two bench lines)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04al; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_render_ws.py tests/test_batch_independence.py tests/test_gpu_kernels.py tests/test_k8.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; tail -5 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c2 -o run -- python3 bench.py --steps 50 --no-cpu-baseline > $O/c2_prof.json 2>/dev/null || exit 2
f=$(find $O/prof_c2 -name '*kernel_stats.csv' | head -1); cp $f $O/c2_kernel_stats.csv
find $O/prof_c2 -type f ! -name '*kernel_stats.csv' -delete
grep -E "ray_order|render_" $O/c2_kernel_stats.csv | cut -c1-160
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --no-cpu-baseline > $O/c2_$i.json 2>/dev/null || exit 3
  python -c "import json; a=json.load(open('$O/c2_$i.json')); print('c2', a['value'], a['ms_per_step'], a['roofline']['kernel_ms'])"
done
