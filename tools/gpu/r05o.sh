#!/bin/bash
# round 5: RCCL world-1 test (verbose), then AMP / ADVICE fixes, expert-parallel suite
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05o; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_rccl_world1.py -v -s -m gpu --timeout 380 --timeout-method thread 2>&1 | tee $O/rccl.log || exit 1
timeout -k 10 600 python -u -m pytest tests/test_amp.py tests/test_expert_parallel.py -v -m gpu --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 2
