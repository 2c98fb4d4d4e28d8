#!/bin/bash
# SQ/TCC/GRBM counter passes on the fused render kernel (one counter group per rocprofv3 run, no
# tracing domains combined with --pmc).  Usage: tools/pmc_render.sh TAG [bench args...]
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-dev}; shift
ARGS=${@:-"--steps 5 --warmup 2 --no-cpu-baseline"}
mkdir -p gpurun_out/pmc_$TAG
i=0
for CTRS in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" \
            "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_WAIT_INST_LDS" \
            "SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_RD" \
            "TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $CTRS --output-format csv -d gpurun_out/pmc_$TAG/p$i -o run -- python3 bench.py $ARGS \
      > gpurun_out/pmc_$TAG/p$i.log 2>&1 || { echo "pass $i failed: $CTRS"; exit 1; }
done
echo "pmc passes done"
