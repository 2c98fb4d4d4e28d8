#!/bin/bash
# round 6: the standalone table-gradient scatter (acn_hashgrid_bwd, the meta query step) -- LDS-merged coarse
# levels (3 / 6) and points per lane (8 / 32) against the default (16, no merge): meta A/B with kernel summaries
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06ah; mkdir -p $O
for rep in 1 2; do
  for v in default m3 m6 p32 p8; do
    if [ $v = default ]; then unset ACNERF_LIB; else export ACNERF_LIB=build_variants/libacnerf_$v.so; fi
    timeout -k 10 300 python -u bench.py --workload meta --no-cpu-baseline > $O/meta_${v}_$rep.json 2> $O/meta_${v}_$rep.err || exit 2
  done
done
unset ACNERF_LIB
for v in default m6 p32; do
  if [ $v = default ]; then unset ACNERF_LIB; else export ACNERF_LIB=build_variants/libacnerf_$v.so; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$v -o run -- python3 bench.py --workload meta --no-cpu-baseline --steps 3 > $O/prof_$v.log 2>&1 || exit 3
  find $O/prof_$v -type f ! -name '*kernel_stats.csv' -delete
done
unset ACNERF_LIB
