#!/bin/bash
# One GPU session: tests, smoke, bench, rocprof kernel stats, PMC passes.  Every GPU step has its
# own time limit and the steps are chained with && (stop at the first failure).
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-r01}
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -q -m gpu -p no:cacheprovider > gpurun_out/pytest_gpu_$TAG.log 2>&1 \
&& timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 \
&& timeout -k 10 300 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err \
&& timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/prof_$TAG.log 2>&1 \
&& timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch_$TAG -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/pmc_fetch_$TAG.log 2>&1 \
&& timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write_$TAG -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/pmc_write_$TAG.log 2>&1
echo "gpu_round exit=$?"
