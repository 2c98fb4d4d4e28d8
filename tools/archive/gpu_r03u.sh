#!/bin/bash
# routed step without autograd in the shared part + padding folded into the scatter: tests; then the hash-grid
# backward points-per-lane (ACN_HASH_BWD_PPL) sweep on the meta-like micro and the C5 step
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03u
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_train.py tests/test_graph_gpu.py tests/test_expert_parallel.py tests/test_loss_gpu.py -m gpu -q \
  --timeout 240 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|ERROR" $O/pytest.log | head -20; tail -2 $O/pytest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for v in default ppl8 ppl32 ppl48; do
  L=adaptive_city_nerf_amd/libacnerf.so; [ $v = default ] || L=build_variants/libacnerf_$v.so
  ACNERF_LIB=$L timeout -k 10 200 python -u tools/micro/hash_bwd.py 2>&1 | grep -v amdgpu.ids | tail -1 || exit 1
  ACNERF_LIB=$L timeout -k 10 300 python -u bench.py --workload c5 --no-cpu-baseline 2>/dev/null > $O/c5_$v.json || exit 1
  python3 -c "import json; d=json.load(open('$O/c5_$v.json')); print('  c5', d['ms_per_step'], 'adam', d['roofline']['kernel_ms'], 'hash bwd', d['roofline']['secondary'].get('kernel_ms'))"
done
