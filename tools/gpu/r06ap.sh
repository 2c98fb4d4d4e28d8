#!/bin/bash
# round 6 (resumed): producer/consumer pair-list MLP backward (mlp_bwd_dw_pairs_pc_kernel, ACN_DW_PAIRS_PC) in the
# C5 step: routed-training parity tests (fixture replays, fused-glue bitwise, AMP, expert-parallel), C5 A/B
# against pairs0 (mlp_bwd_dw_pairs_kernel), rotated, and the C5 kernel summary
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06ap; mkdir -p $O
unset ACNERF_LIB
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_train.py \
  tests/test_routed_glue.py tests/test_amp.py tests/test_determinism_gpu.py tests/test_expert_parallel.py \
  tests/test_k8.py tests/test_graph_gpu.py > $O/tests.txt 2>&1 || exit 1
for order in "default pairs0" "pairs0 default" "default pairs0"; do
  rep=$((rep+1))
  for v in $order; do
    if [ $v = default ]; then unset ACNERF_LIB; else export ACNERF_LIB=build_variants/libacnerf_$v.so; fi
    timeout -k 10 300 python -u bench.py --workload c5 --no-cpu-baseline > $O/c5_${v}_$rep.json 2> $O/c5_${v}_$rep.err || exit 3
  done
done
unset ACNERF_LIB
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c5 -o run -- python3 bench.py --workload c5 --no-cpu-baseline > $O/prof_c5.log 2>&1 || exit 5
find $O/prof_c5 -type f ! -name '*kernel_stats.csv' -delete
