#!/bin/bash
# round 4, first call: counters of the render kernels on the round-3 build (C2 render_kernel, C3 / C4-S96
# render_slots_kernel) and the C3 / C4-S96 lines with their CPU baselines
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04a
mkdir -p $O
bash tools/pmc_r04.sh c2 --steps 5 --warmup 2 --no-cpu-baseline || exit 1
bash tools/pmc_r04.sh c3 --workload c3 --steps 5 --warmup 2 --no-cpu-baseline || exit 2
bash tools/pmc_r04.sh c4s96 --workload c4 --samples 96 --steps 2 --warmup 1 --no-cpu-baseline || exit 3
timeout -k 10 300 python -u bench.py --workload c3 --steps 100 > $O/bench_c3.json 2> $O/bench_c3.err || { echo "c3 failed"; tail -5 $O/bench_c3.err; exit 4; }
cut -c1-300 $O/bench_c3.json
timeout -k 10 300 python -u bench.py --workload c4 --samples 96 --steps 5 > $O/bench_c4s96.json 2> $O/bench_c4s96.err || { echo "c4 failed"; tail -5 $O/bench_c4s96.err; exit 5; }
cut -c1-300 $O/bench_c4s96.json
echo "r04a done"
