#!/bin/bash
# round 5: RCCL world-1 test, AMP / EP suites; C3 timing of the routed work-shared render variants
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05p; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_rccl_world1.py -v -s -m gpu --timeout 380 --timeout-method thread > $O/rccl.log 2>&1
timeout -k 10 600 python -u -m pytest tests/test_amp.py tests/test_expert_parallel.py -v -m gpu --timeout 300 --timeout-method thread > $O/tests.log 2>&1
timeout -k 10 200 python -u bench.py --workload c3 --no-cpu-baseline > $O/c3_slots.json 2>$O/c3_slots.err || exit 3
for v in rws_l2call rws_ldsonly; do
  ACNERF_LIB=build_variants/libacnerf_$v.so timeout -k 10 200 python -u bench.py --workload c3 --no-cpu-baseline > $O/c3_$v.json 2>$O/c3_$v.err || exit 4
done
