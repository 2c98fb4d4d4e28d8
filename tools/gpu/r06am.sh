#!/bin/bash
# round 6 (resumed): (1) the no-save MLP forward on vector h0 / SH loads (fwdv = ACN_FWD_VLOAD=1): training-MLP
# parity tests on that library, meta A/B; (2) the standalone table-gradient scatter of the meta step (r06ah's
# variants: LDS-merged coarse levels m3 / m6, points per lane p32 / p8 against 16)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06am; mkdir -p $O
export ACNERF_LIB=build_variants/libacnerf_fwdv.so
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_mlp_train_gpu.py \
  tests/test_meta_gpu.py tests/test_determinism_gpu.py tests/test_amp.py > $O/tests_fwdv.txt 2>&1 || exit 1
for rep in 1 2; do
  for v in default fwdv m3 m6 p32 p8; do
    if [ $v = default ]; then unset ACNERF_LIB; else export ACNERF_LIB=build_variants/libacnerf_$v.so; fi
    timeout -k 10 300 python -u bench.py --workload meta --no-cpu-baseline > $O/meta_${v}_$rep.json 2> $O/meta_${v}_$rep.err || exit 2
  done
done
for v in fwdv m6 p32; do
  export ACNERF_LIB=build_variants/libacnerf_$v.so
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_meta_$v -o run -- python3 bench.py --workload meta --no-cpu-baseline --steps 3 > $O/prof_meta_$v.log 2>&1 || exit 4
  find $O/prof_meta_$v -type f ! -name '*kernel_stats.csv' -delete
done
