#!/bin/bash
# round 5: LDS counters of the meta step's fused MLP backward (is mlp_bwd_dw_pc_kernel LDS-bound?)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05ag; mkdir -p $O
timeout -s KILL 240 rocprofv3 --pmc SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $O/lds -o run -- python3 bench.py --workload meta --steps 3 --warmup 1 --no-cpu-baseline > $O/lds.log 2>&1 || { tail -5 $O/lds.log; exit 1; }
python tools/pmc_filter.py $O mlp_bwd_dw_pc_kernel
