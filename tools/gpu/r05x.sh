#!/bin/bash
# round 5: the operand fence in the training MLP (mlp_train.hip) -- cost on the meta step and run-to-run stability
# of the fused forward / backward with the fence, without its scheduling barriers, without its nops, and without it
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05x; mkdir -p $O
for v in default mlpsb0 mlpnopad mlpoff; do
  if [ $v = default ]; then unset ACNERF_LIB; else export ACNERF_LIB=build_variants/libacnerf_$v.so; fi
  ACN_DET_REPS=100 timeout -k 10 300 python -u -m pytest tests/test_determinism_gpu.py -k "training_mlp and fp16x3" -q -m gpu --timeout 280 --timeout-method thread > $O/det_$v.log 2>&1
  echo "$v determinism rc=$? $(tail -1 $O/det_$v.log)"
  timeout -k 10 300 python -u bench.py --workload meta --steps 10 --warmup 3 --no-cpu-baseline > $O/meta_$v.json 2>$O/meta_$v.err || { echo "meta $v failed"; tail -3 $O/meta_$v.err; exit 1; }
  python -c "import json;d=json.load(open('$O/meta_$v.json'));print('meta $v', d['ms_per_step'], d['roofline']['kernel_ms'])"
done
