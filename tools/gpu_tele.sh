#!/bin/bash
# telescoped table norm: routed-step GPU tests, then C5 with / without it (A/B)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_train.py tests/test_graph_gpu.py tests/test_expert_parallel.py -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/pt_tele.log 2>&1
rc=$?; tail -1 gpurun_out/pt_tele.log; [ $rc = 0 ] || exit $rc
: > gpurun_out/ab_tele.txt
for v in 1 0 1 0; do
  ACN_TELE_NORM=$v timeout -k 10 200 python bench.py --workload c5 --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/abt_$v.json 2> gpurun_out/abt_$v.err || exit 1
  python -c "import json; d=json.loads(open('gpurun_out/abt_$v.json').read().strip().splitlines()[-1]); print('tele=$v', d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline'].get('secondary',{}).get('kernel_ms'), d['val_psnr_db'])" >> gpurun_out/ab_tele.txt
done
cat gpurun_out/ab_tele.txt
