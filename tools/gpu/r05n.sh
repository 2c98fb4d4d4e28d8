#!/bin/bash
# round 5: expert-parallel tests (planned exchange) + C4 S=96 expert layout line
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05n; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_expert_parallel.py -x -q -m gpu --timeout 300 --timeout-method thread > $O/ep_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --workload c4 --samples 96 --steps 5 --layout expert --no-cpu-baseline > $O/c4s96_expert.json 2>$O/c4e.err || exit 2
