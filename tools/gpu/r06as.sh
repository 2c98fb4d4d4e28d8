#!/bin/bash
# round 6 (resumed): the optimizer passes on global-address-space loads / stores (ACN_ADAM_GLOBAL; the descriptor
# pointers gave flat_* instructions, whose waits cannot be partial): Adam / training parity tests, C5 and meta A/B
# against the flat variant, rotated, and the C5 kernel summary
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06as; mkdir -p $O
unset ACNERF_LIB
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_train.py \
  tests/test_routed_glue.py tests/test_amp.py tests/test_graph_gpu.py tests/test_meta_gpu.py tests/test_expert_parallel.py \
  tests/test_rccl_world1.py > $O/tests.txt 2>&1 || exit 1
for order in "default flat" "flat default" "default flat"; do
  rep=$((rep+1))
  for v in $order; do
    if [ $v = default ]; then unset ACNERF_LIB; else export ACNERF_LIB=build_variants/libacnerf_$v.so; fi
    timeout -k 10 300 python -u bench.py --workload c5 --no-cpu-baseline > $O/c5_${v}_$rep.json 2> $O/c5_${v}_$rep.err || exit 3
  done
done
for v in default flat; do
  if [ $v = default ]; then unset ACNERF_LIB; else export ACNERF_LIB=build_variants/libacnerf_$v.so; fi
  timeout -k 10 300 python -u bench.py --workload meta --no-cpu-baseline > $O/meta_${v}.json 2> $O/meta_${v}.err || exit 4
done
unset ACNERF_LIB
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c5 -o run -- python3 bench.py --workload c5 --no-cpu-baseline > $O/prof_c5.log 2>&1 || exit 5
find $O/prof_c5 -type f ! -name '*kernel_stats.csv' -delete
