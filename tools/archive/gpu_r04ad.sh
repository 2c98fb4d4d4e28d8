#!/bin/bash
# producer / consumer balance of the fused MLP backward (tools/micro/mlp_bwd_roles.py on diagnostic builds)
set -o pipefail
export TMPDIR=/tmp
for v in base mlp_nodw mlp_noprod amp_nodw amp_noprod; do
  if [ $v = base ]; then unset ACNERF_LIB; else export ACNERF_LIB=$PWD/build_variants/libacnerf_$v.so; fi
  timeout -k 10 120 python -u tools/micro/mlp_bwd_roles.py $v 2>&1 | grep bwd_dw || exit 1
done
