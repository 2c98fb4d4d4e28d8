#!/bin/bash
# work-shared round in render_slots_kernel: bitwise tests + routed suites, then C3 / C4-S96 A/B against the
# per-wave round (slotsws0), alternating
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04am; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_render_ws.py tests/test_batch_independence.py tests/test_k8.py tests/test_gpu_kernels.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; tail -4 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for v in base slotsws0 base slotsws0; do
  lib=adaptive_city_nerf_amd/libacnerf.so; [ $v = base ] || lib=build_variants/libacnerf_$v.so
  for w in "c3:--workload c3" "c4s96:--workload c4 --samples 96"; do
    tag=${w%%:*}; args=${w#*:}
    ACNERF_LIB=$lib timeout -k 10 200 python -u bench.py --no-cpu-baseline $args > $O/${tag}_$v.json 2>$O/${tag}_$v.err || { tail -3 $O/${tag}_$v.err; exit 3; }
    python -c "import json; a=json.load(open('$O/${tag}_$v.json')); print('$tag $v', a['value'], a['ms_per_step'], a['roofline'].get('kernel_ms'))"
  done
done
