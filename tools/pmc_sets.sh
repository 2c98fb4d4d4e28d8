#!/bin/bash
# Run rocprofv3 --pmc passes (one counter set per run) over bench.py.
# Usage: tools/pmc_sets.sh OUTDIR "SET1" "SET2" ...   (ACNERF_LIB may select a variant build)
set -o pipefail
export TMPDIR=/tmp
OUT=$1; shift
mkdir -p $OUT
i=0
for CTRS in "$@"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $CTRS --output-format csv -d $OUT/p$i -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline \
      > $OUT/p$i.log 2>&1 || { echo "pass $i failed: $CTRS"; exit 1; }
done
echo "pmc sets done: $OUT"
