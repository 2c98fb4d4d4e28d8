#!/bin/bash
# Round-end refresh: full GPU suite + smoke, then every workload's bench line (with its CPU baseline)
# and kernel-stats profiles of the training workloads.  Steps chained with &&, each under its own limit.
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-all}
mkdir -p gpurun_out
keep_stats() { find "$1" -type f ! -name '*kernel_stats.csv' -delete; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_$TAG.log 2>&1 \
&& timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 \
&& for w in c2 c3 c4 c5 occ meta data clusters; do
     extra=""; [ $w = meta ] && extra="--steps 5 --warmup 2"
     timeout -k 10 300 python -u bench.py --workload $w $extra > gpurun_out/bench_${w}_$TAG.json 2> gpurun_out/bench_${w}_$TAG.err || exit 1
   done \
&& timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c5_$TAG -o run -- python3 bench.py --workload c5 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/prof_c5_$TAG.log 2>&1 && keep_stats gpurun_out/prof_c5_$TAG \
&& timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_meta_$TAG -o run -- python3 bench.py --workload meta --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof_meta_$TAG.log 2>&1 && keep_stats gpurun_out/prof_meta_$TAG \
&& timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c2_$TAG -o run -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/prof_c2_$TAG.log 2>&1 && keep_stats gpurun_out/prof_c2_$TAG
echo "gpu_bench_all exit=$?"
