#!/bin/bash
# round 6 (resumed): MLP backward producers' prefetch (vector loads of h0 / SH / outputs issued ahead of use,
# ACN_DW_PREFETCH) -- training-MLP parity tests, then meta A/B against nopf (the in-place loads) and pfprio
# (prefetch + producers' wave priority raised), the meta kernel summary
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06al; mkdir -p $O
unset ACNERF_LIB
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_mlp_train_gpu.py \
  tests/test_meta_gpu.py tests/test_determinism_gpu.py tests/test_amp.py tests/test_train.py > $O/tests.txt 2>&1 || exit 1
for rep in 1 2; do
  for v in default nopf pfprio; do
    if [ $v = default ]; then unset ACNERF_LIB; else export ACNERF_LIB=build_variants/libacnerf_$v.so; fi
    timeout -k 10 300 python -u bench.py --workload meta --no-cpu-baseline > $O/meta_${v}_$rep.json 2> $O/meta_${v}_$rep.err || exit 2
  done
done
for v in default pfprio; do
  if [ $v = default ]; then unset ACNERF_LIB; else export ACNERF_LIB=build_variants/libacnerf_$v.so; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_meta_$v -o run -- python3 bench.py --workload meta --no-cpu-baseline --steps 3 > $O/prof_meta_$v.log 2>&1 || exit 4
  find $O/prof_meta_$v -type f ! -name '*kernel_stats.csv' -delete
done
