#!/bin/bash
# the split routed render (ACN_SPLIT_ROUTED=1) rebuilt with the round-3 "codegen hazard" form
# (ACN_SINGLE_EXSEL=0: runtime-indexed ExpertMeta + LDS weights), with and without the layer_x3 pad
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04r; mkdir -p $O
for v in split_exsel0 split_exsel0_nop0; do
  for rep in 1 2; do
    ACNERF_LIB=$PWD/build_variants/libacnerf_$v.so timeout -k 10 300 python -u -m pytest tests/test_k8.py -m gpu -k split_routed \
        -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/${v}_$rep.log 2>&1
    echo "$v rep $rep rc=$? $(tail -1 $O/${v}_$rep.log)"
  done
done
