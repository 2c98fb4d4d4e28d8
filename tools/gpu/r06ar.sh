#!/bin/bash
# round 6 (resumed): fp16x3 layer products with the output tiles' MFMA chains interleaved (ACN_MLP_ILV): training
# parity tests, meta / C5 A/B against ilv0, rotated; merged-level count of the meta scatter (sa4 / sa8 vs 6)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06ar; mkdir -p $O
unset ACNERF_LIB
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_mlp_train_gpu.py \
  tests/test_meta_gpu.py tests/test_determinism_gpu.py tests/test_amp.py tests/test_train.py tests/test_routed_glue.py \
  tests/test_k8.py > $O/tests.txt 2>&1 || exit 1
for order in "default ilv0 sa4 sa8" "sa8 sa4 ilv0 default"; do
  rep=$((rep+1))
  for v in $order; do
    if [ $v = default ]; then unset ACNERF_LIB; else export ACNERF_LIB=build_variants/libacnerf_$v.so; fi
    timeout -k 10 300 python -u bench.py --workload meta --no-cpu-baseline > $O/meta_${v}_$rep.json 2> $O/meta_${v}_$rep.err || exit 2
    if [ $v = default ] || [ $v = ilv0 ]; then
      timeout -k 10 300 python -u bench.py --workload c5 --no-cpu-baseline > $O/c5_${v}_$rep.json 2> $O/c5_${v}_$rep.err || exit 3
    fi
  done
done
unset ACNERF_LIB
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_meta -o run -- python3 bench.py --workload meta --no-cpu-baseline --steps 3 > $O/prof_meta.log 2>&1 || exit 4
find $O/prof_meta -type f ! -name '*kernel_stats.csv' -delete
