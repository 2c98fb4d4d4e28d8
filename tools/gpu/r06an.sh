#!/bin/bash
# round 6 (resumed): the meta step's standalone scatter with 6 LDS-merged coarse levels by default
# (ACN_HASH_BWD_MERGE_SA=6): hash / meta / deterministic-scatter tests; meta A/B against sa0 (no merge, before),
# sa6p8 (merge + 8 points per lane) and fwdv (vector loads in the no-save MLP forward), order rotated per rep
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06an; mkdir -p $O
unset ACNERF_LIB
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py \
  tests/test_meta_gpu.py tests/test_hash_det.py tests/test_train.py > $O/tests.txt 2>&1 || exit 1
for order in "default sa0 sa6p8 fwdv" "fwdv sa6p8 sa0 default" "sa0 default fwdv sa6p8"; do
  rep=$((rep+1))
  for v in $order; do
    if [ $v = default ]; then unset ACNERF_LIB; else export ACNERF_LIB=build_variants/libacnerf_$v.so; fi
    timeout -k 10 300 python -u bench.py --workload meta --no-cpu-baseline > $O/meta_${v}_$rep.json 2> $O/meta_${v}_$rep.err || exit 2
  done
done
unset ACNERF_LIB
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_meta -o run -- python3 bench.py --workload meta --no-cpu-baseline --steps 3 > $O/prof_meta.log 2>&1 || exit 4
find $O/prof_meta -type f ! -name '*kernel_stats.csv' -delete
