#!/bin/bash
# Counter passes for one program (round 6: any script, not only bench.py): a kernel-trace / stats run, then one rocprofv3 --pmc
# pass per counter group (FETCH_SIZE takes 3 TCC counters and WRITE_SIZE 2, so each gets its own pass;
# no tracing domain is combined with --pmc).  Every pass runs under its own hard time limit.
# usage: tools/pmc_r06.sh TAG script.py args...     -> gpurun_out/pmc_TAG/{stats,p1..p6}
set -o pipefail
export TMPDIR=/tmp
TAG=$1; shift
ARGS="$@"
O=gpurun_out/pmc_$TAG
mkdir -p $O
timeout -s KILL 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run -- python3 $ARGS \
    > $O/stats.log 2>&1 || { echo "stats pass failed ($TAG)"; tail -5 $O/stats.log; exit 1; }
find $O/stats -type f ! -name '*kernel_stats.csv' -delete
i=0
for CTRS in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" \
            "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_VMEM_RD SQ_INSTS_LDS GRBM_GUI_ACTIVE" \
            "TCC_HIT_sum TCC_MISS_sum" \
            "FETCH_SIZE" \
            "WRITE_SIZE" \
            "TD_TD_BUSY_sum TD_TC_STALL_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 180 rocprofv3 --pmc $CTRS --output-format csv -d $O/p$i -o run -- python3 $ARGS \
      > $O/p$i.log 2>&1 || { echo "pmc pass $i failed ($TAG): $CTRS"; tail -5 $O/p$i.log; exit 1; }
  find $O/p$i -type f ! -name '*counter_collection.csv' -delete
done
echo "pmc $TAG done"
