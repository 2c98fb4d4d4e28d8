#!/bin/bash
# round 6 (resumed), closing run on the final build: full GPU suite + smoke, every bench line (C2 with its CPU
# baseline), the C2 / C5 / meta kernel summaries
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06aq; mkdir -p $O
unset ACNERF_LIB
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_suite.txt 2>&1 || exit 1
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || exit 2
timeout -k 10 400 python -u bench.py > $O/bench_c2.json 2> $O/bench_c2.err || exit 3
timeout -k 10 200 python -u bench.py --workload c3 --no-cpu-baseline > $O/bench_c3.json 2> $O/bench_c3.err || exit 4
timeout -k 10 300 python -u bench.py --workload c4 --samples 96 --steps 5 --no-cpu-baseline > $O/bench_c4s96.json 2> $O/bench_c4s96.err || exit 5
timeout -k 10 300 python -u bench.py --workload c4 --steps 3 --no-cpu-baseline > $O/bench_c4.json 2> $O/bench_c4.err || exit 5
timeout -k 10 300 python -u bench.py --workload c4 --samples 96 --steps 5 --layout expert --no-cpu-baseline > $O/bench_c4s96_expert.json 2> $O/bench_c4s96_expert.err || exit 6
timeout -k 10 300 python -u bench.py --workload c5 > $O/bench_c5.json 2> $O/bench_c5.err || exit 7
timeout -k 10 300 python -u bench.py --workload meta > $O/bench_meta.json 2> $O/bench_meta.err || exit 8
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c2 -o run -- python3 bench.py --no-cpu-baseline > $O/prof_c2.log 2>&1 || exit 9
find $O/prof_c2 -type f ! -name '*kernel_stats.csv' -delete
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c5 -o run -- python3 bench.py --workload c5 --no-cpu-baseline > $O/prof_c5.log 2>&1 || exit 10
find $O/prof_c5 -type f ! -name '*kernel_stats.csv' -delete
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_meta -o run -- python3 bench.py --workload meta --no-cpu-baseline --steps 3 > $O/prof_meta.log 2>&1 || exit 11
find $O/prof_meta -type f ! -name '*kernel_stats.csv' -delete
# the pair-list producer/consumer backward (unpipelined contraction) against mlp_bwd_dw_pairs_kernel, rotated
for order in "pairs0 default" "default pairs0"; do
  rep=$((rep+1))
  for v in $order; do
    if [ $v = default ]; then unset ACNERF_LIB; else export ACNERF_LIB=build_variants/libacnerf_$v.so; fi
    timeout -k 10 300 python -u bench.py --workload c5 --no-cpu-baseline > $O/c5ab_${v}_$rep.json 2> $O/c5ab_${v}_$rep.err || exit 12
  done
done
