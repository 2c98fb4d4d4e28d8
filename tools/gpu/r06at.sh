#!/bin/bash
# round 6 (resumed): 16-B bias reads in the fp16x3 layer epilogue (ACN_MLP_BIASV): full GPU suite + smoke on this
# build, meta A/B against biasv0 (rotated), the C2 / C5 / meta lines and the meta kernel summary
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06at; mkdir -p $O
unset ACNERF_LIB
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_suite.txt 2>&1 || exit 1
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || exit 2
for order in "default biasv0" "biasv0 default"; do
  rep=$((rep+1))
  for v in $order; do
    if [ $v = default ]; then unset ACNERF_LIB; else export ACNERF_LIB=build_variants/libacnerf_$v.so; fi
    timeout -k 10 300 python -u bench.py --workload meta --no-cpu-baseline > $O/meta_${v}_$rep.json 2> $O/meta_${v}_$rep.err || exit 3
  done
done
unset ACNERF_LIB
timeout -k 10 400 python -u bench.py > $O/bench_c2.json 2> $O/bench_c2.err || exit 4
timeout -k 10 300 python -u bench.py --workload c5 > $O/bench_c5.json 2> $O/bench_c5.err || exit 5
timeout -k 10 300 python -u bench.py --workload meta > $O/bench_meta.json 2> $O/bench_meta.err || exit 6
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_meta -o run -- python3 bench.py --workload meta --no-cpu-baseline --steps 3 > $O/prof_meta.log 2>&1 || exit 7
find $O/prof_meta -type f ! -name '*kernel_stats.csv' -delete
