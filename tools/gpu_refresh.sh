#!/bin/bash
# Round-end refresh of the render lines: full GPU suite + smoke, the render workloads' bench lines and
# kernel-stats profiles of C3 / C4.  Steps chained with &&, each under its own limit.
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-refresh}
mkdir -p gpurun_out
keep_stats() { find "$1" -type f ! -name '*kernel_stats.csv' -delete; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_$TAG.log 2>&1 \
&& timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 \
&& for w in c2 c3 c4; do
     timeout -k 10 300 python -u bench.py --workload $w > gpurun_out/bench_${w}_$TAG.json 2> gpurun_out/bench_${w}_$TAG.err || exit 1
   done \
&& timeout -k 10 300 python -u bench.py --workload c4 --samples 96 > gpurun_out/bench_c4s96_$TAG.json 2> gpurun_out/bench_c4s96_$TAG.err \
&& timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c3_$TAG -o run -- python3 bench.py --workload c3 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/prof_c3_$TAG.log 2>&1 && keep_stats gpurun_out/prof_c3_$TAG \
&& timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c4_$TAG -o run -- python3 bench.py --workload c4 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof_c4_$TAG.log 2>&1 && keep_stats gpurun_out/prof_c4_$TAG
rc=$?
[ $rc = 0 ] && ACN_TRACE_MARK=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trace_c2_$TAG -o run -- python3 bench.py --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/trace_c2_$TAG.log 2>&1 \
  && python tools/trace_busy.py gpurun_out/trace_c2_$TAG 50 > gpurun_out/trace_c2_$TAG.txt; rc=$?
echo "gpu_refresh exit=$rc"
