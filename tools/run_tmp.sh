set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu_prof.sh c2r02b "--steps 20 --warmup 3" &&
bash tools/pmc_sets.sh gpurun_out/pmc_c2r02b "TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE" "WRITE_SIZE" \
   "SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD" \
   "TD_TD_BUSY_sum TD_TC_STALL_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum" &&
bash tools/gpu_prof.sh c5r02b "--workload c5 --steps 20 --warmup 5" &&
bash tools/pmc_c5.sh &&
bash tools/gpu_prof.sh metar02b "--workload meta --steps 3 --warmup 1"
echo rc=$?
