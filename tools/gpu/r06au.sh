#!/bin/bash
# round 6 (resumed): fp16x3 layers read the next k-step's A operands ahead (ACN_MLP_KPIPE): full GPU suite + smoke on
# this build, meta / C5 A/B against kpipe0 (rotated), the C2 / C5 / meta lines and the meta kernel summary
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06au; mkdir -p $O
unset ACNERF_LIB
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_suite.txt 2>&1 || exit 1
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || exit 2
for order in "default kpipe0" "kpipe0 default"; do
  rep=$((rep+1))
  for v in $order; do
    if [ $v = default ]; then unset ACNERF_LIB; else export ACNERF_LIB=build_variants/libacnerf_$v.so; fi
    timeout -k 10 300 python -u bench.py --workload meta --no-cpu-baseline > $O/meta_${v}_$rep.json 2> $O/meta_${v}_$rep.err || exit 3
    timeout -k 10 300 python -u bench.py --workload c5 --no-cpu-baseline > $O/c5_${v}_$rep.json 2> $O/c5_${v}_$rep.err || exit 4
  done
done
unset ACNERF_LIB
timeout -k 10 400 python -u bench.py > $O/bench_c2.json 2> $O/bench_c2.err || exit 5
timeout -k 10 300 python -u bench.py --workload meta > $O/bench_meta.json 2> $O/bench_meta.err || exit 6
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_meta -o run -- python3 bench.py --workload meta --no-cpu-baseline --steps 3 > $O/prof_meta.log 2>&1 || exit 7
find $O/prof_meta -type f ! -name '*kernel_stats.csv' -delete
