#!/bin/bash
# round 6 (resumed): level-major hash forward (hashgrid_fwd_f2_lm / hashgrid_fwd_pairs_lm) and the MLP backward's
# stage-free barrier at the round head (ACN_DW_HEADSYNC): targeted parity tests, then meta / C5 A/B against the
# variants that undo each change, and the meta kernel summary
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06aj; mkdir -p $O
unset ACNERF_LIB
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py \
  tests/test_mlp_train_gpu.py tests/test_meta_gpu.py tests/test_train.py tests/test_routed_glue.py \
  tests/test_determinism_gpu.py tests/test_amp.py > $O/tests.txt 2>&1 || exit 1
for rep in 1 2; do
  for v in default mlpend fwdpl; do
    if [ $v = default ]; then unset ACNERF_LIB; else export ACNERF_LIB=build_variants/libacnerf_$v.so; fi
    timeout -k 10 300 python -u bench.py --workload meta --no-cpu-baseline > $O/meta_${v}_$rep.json 2> $O/meta_${v}_$rep.err || exit 2
  done
  for v in default fwdpl; do
    if [ $v = default ]; then unset ACNERF_LIB; else export ACNERF_LIB=build_variants/libacnerf_$v.so; fi
    timeout -k 10 300 python -u bench.py --workload c5 --no-cpu-baseline > $O/c5_${v}_$rep.json 2> $O/c5_${v}_$rep.err || exit 3
  done
done
unset ACNERF_LIB
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_meta -o run -- python3 bench.py --workload meta --no-cpu-baseline --steps 3 > $O/prof_meta.log 2>&1 || exit 4
find $O/prof_meta -type f ! -name '*kernel_stats.csv' -delete
export ACNERF_LIB=build_variants/libacnerf_fwdpl.so
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_meta_fwdpl -o run -- python3 bench.py --workload meta --no-cpu-baseline --steps 3 > $O/prof_meta_fwdpl.log 2>&1 || exit 5
find $O/prof_meta_fwdpl -type f ! -name '*kernel_stats.csv' -delete
