#!/bin/bash
# Refresh of the training / pipeline lines: meta, occ, data, clusters bench lines (with CPU baselines),
# meta rocprof kernel stats.  Steps chained with &&, each under its own limit.
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-refresh2}
mkdir -p gpurun_out
keep_stats() { find "$1" -type f ! -name '*kernel_stats.csv' -delete; }
for w in meta occ data clusters; do
  extra=""; [ $w = meta ] && extra="--steps 5 --warmup 2"
  timeout -k 10 300 python -u bench.py --workload $w $extra > gpurun_out/bench_${w}_$TAG.json 2> gpurun_out/bench_${w}_$TAG.err || { echo "bench $w failed"; exit 1; }
done \
&& timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_meta_$TAG -o run -- python3 bench.py --workload meta --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof_meta_$TAG.log 2>&1 && keep_stats gpurun_out/prof_meta_$TAG
echo "gpu_refresh2 exit=$?"
