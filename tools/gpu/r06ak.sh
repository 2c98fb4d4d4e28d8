#!/bin/bash
# round 6 (resumed): MLP backward wave priority (ACN_DW_PRIO 1 producers / 2 consumers raised) and the stage-free
# barrier placement (mlpend = round end) on the meta step; the new hash-forward parity tests on the default build
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06ak; mkdir -p $O
unset ACNERF_LIB
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k hashgrid > $O/tests.txt 2>&1 || exit 1
for rep in 1 2; do
  for v in default prio1 prio2 mlpend; do
    if [ $v = default ]; then unset ACNERF_LIB; else export ACNERF_LIB=build_variants/libacnerf_$v.so; fi
    timeout -k 10 300 python -u bench.py --workload meta --no-cpu-baseline > $O/meta_${v}_$rep.json 2> $O/meta_${v}_$rep.err || exit 2
  done
done
for v in prio1 prio2; do
  export ACNERF_LIB=build_variants/libacnerf_$v.so
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_meta_$v -o run -- python3 bench.py --workload meta --no-cpu-baseline --steps 3 > $O/prof_meta_$v.log 2>&1 || exit 4
  find $O/prof_meta_$v -type f ! -name '*kernel_stats.csv' -delete
done
