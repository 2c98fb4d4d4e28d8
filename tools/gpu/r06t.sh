#!/bin/bash
# round 6: depth-tiled record order in the expert-parallel renderer (acn_routed_*_tiled) -- EP tests, every rank of
# the one-expert-per-GPU C4 layout in both orders, counter passes of the busiest rank, the --layout expert line
# with and without tiles
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06t; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q -m gpu --timeout 600 --timeout-method thread tests/test_expert_parallel.py tests/test_rccl_world1.py > $O/ep_tests.txt 2>&1 || exit 1
timeout -k 10 300 python -u tools/ep_owner_rank.py --expert -1 > $O/ep_ranks_tiled.jsonl 2> $O/ep_ranks_tiled.err || exit 2
timeout -k 10 300 python -u tools/ep_owner_rank.py --expert -1 --order sample > $O/ep_ranks_sample.jsonl 2> $O/ep_ranks_sample.err || exit 2
timeout -k 10 600 bash tools/pmc_r06.sh ep_owner_tiled tools/ep_owner_rank.py > $O/pmc_ep.log 2>&1 || exit 3
for rep in 1 2; do
  timeout -k 10 300 python -u bench.py --workload c4 --samples 96 --steps 5 --layout expert --no-cpu-baseline > $O/expert_t32_$rep.json 2> $O/expert_t32_$rep.err || exit 4
  ACN_EP_TILE=0 timeout -k 10 300 python -u bench.py --workload c4 --samples 96 --steps 5 --layout expert --no-cpu-baseline > $O/expert_t0_$rep.json 2> $O/expert_t0_$rep.err || exit 4
done
