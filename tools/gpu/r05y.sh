#!/bin/bash
# round 5: long run-to-run stress of the training MLP (fp16x3 and use_amp, meta batch) with and without the fence
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05y; mkdir -p $O
for v in mlpoff default; do
  if [ $v = default ]; then unset ACNERF_LIB; else export ACNERF_LIB=build_variants/libacnerf_$v.so; fi
  ACN_DET_REPS=4000 timeout -k 10 500 python -u -m pytest tests/test_determinism_gpu.py -k "training_mlp and 362666 and (fp16x3 or amp)" -q -m gpu --timeout 480 --timeout-method thread > $O/det_$v.log 2>&1
  echo "$v determinism rc=$? $(tail -1 $O/det_$v.log)"
done
