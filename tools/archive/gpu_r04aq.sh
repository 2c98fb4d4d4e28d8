#!/bin/bash
# work-shared occupancy render: occupancy tests, bitwise check against occ_render_kernel, occ bench A/B
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04aq; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_occ_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/micro/occ_ws_check.py $O/occ_ws.npz > $O/chk1.log 2>&1 || { tail -5 $O/chk1.log; exit 2; }
ACNERF_LIB=build_variants/libacnerf_occws0.so timeout -k 10 200 python -u tools/micro/occ_ws_check.py $O/occ_old.npz > $O/chk2.log 2>&1 || { tail -5 $O/chk2.log; exit 3; }
python tools/micro/occ_ws_check.py --compare $O/occ_ws.npz $O/occ_old.npz || exit 4
for v in base occws0 base occws0; do
  lib=adaptive_city_nerf_amd/libacnerf.so; [ $v = base ] || lib=build_variants/libacnerf_$v.so
  ACNERF_LIB=$lib timeout -k 10 200 python -u bench.py --workload occ --no-cpu-baseline > $O/occ_$v.json 2>$O/occ_$v.err || { tail -3 $O/occ_$v.err; exit 5; }
  python -c "import json; a=json.loads(open('$O/occ_$v.json').read().strip().splitlines()[-1]); print('occ $v', a['value'], a['ms_per_step'], a['roofline'].get('kernel_ms'))"
done
