#!/bin/bash
# fused background head in the routed C5 step: training GPU tests, then C5 with / without it (A/B)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_train.py tests/test_graph_gpu.py tests/test_expert_parallel.py -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/pt_bg.log 2>&1
rc=$?; tail -1 gpurun_out/pt_bg.log; [ $rc = 0 ] || exit $rc
: > gpurun_out/ab_bg.txt
for v in 1 0 1 0; do
  ACN_FUSED_BG=$v timeout -k 10 200 python bench.py --workload c5 --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/abb_$v.json 2> gpurun_out/abb_$v.err || exit 1
  python -c "import json; d=json.loads(open('gpurun_out/abb_$v.json').read().strip().splitlines()[-1]); print('fused_bg=$v', d['ms_per_step'], d['roofline']['kernel_ms'], d['val_psnr_db']['after'])" >> gpurun_out/ab_bg.txt
done
cat gpurun_out/ab_bg.txt
