#!/bin/bash
# HBM counters of one bench workload's kernels: one rocprofv3 --pmc pass per counter (FETCH_SIZE uses
# 3 TCC counters, WRITE_SIZE 2: they cannot share a pass), each pass under its own hard time limit.
# usage: tools/pmc_kernel.sh WORKLOAD   -> gpurun_out/pmc_WORKLOAD/{fetch,write}/...
set -o pipefail
export TMPDIR=/tmp
W=$1
mkdir -p gpurun_out/pmc_$W
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_$W/fetch -o run --output-format csv -- python3 bench.py --workload $W --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_$W/fetch.log 2>&1 \
&& timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_$W/write -o run --output-format csv -- python3 bench.py --workload $W --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_$W/write.log 2>&1
echo "pmc $W exit=$?"
