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
&& tools/pmc_sets.sh gpurun_out/pmc_$TAG "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_VMEM_RD" "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum" "TD_TD_BUSY_sum TD_TC_STALL_sum" "TCC_HIT_sum TCC_MISS_sum" > gpurun_out/pmc_$TAG.log 2>&1
echo "gpu_round exit=$?"
