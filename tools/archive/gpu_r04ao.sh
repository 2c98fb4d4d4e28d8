#!/bin/bash
# render_dq_kernel (band queues of rays, workgroup-shared tiles): bitwise tests + render suites, then the C2 A/B
# against render_ws_kernel (dq0) and other live-ray caps, alternating
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04ao; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_render_ws.py tests/test_batch_independence.py tests/test_gpu_kernels.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; tail -4 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for v in base dq0 dq8 dq14 base dq0 dq8 dq14; do
  lib=adaptive_city_nerf_amd/libacnerf.so; [ $v = base ] || lib=build_variants/libacnerf_$v.so
  ACNERF_LIB=$lib timeout -k 10 200 python -u bench.py --no-cpu-baseline > $O/c2_$v.json 2>$O/c2_$v.err || { tail -3 $O/c2_$v.err; exit 3; }
  python -c "import json; a=json.load(open('$O/c2_$v.json')); print('c2 $v', a['value'], a['ms_per_step'], a['roofline'].get('kernel_ms'))"
done
