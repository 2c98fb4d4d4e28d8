#!/bin/bash
# round 6: one rank of the one-expert-per-GPU C4 layout: every rank's owner kernel timed, then
# a kernel-trace summary and the counter passes of the busiest rank
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06m; mkdir -p $O
timeout -k 10 300 python -u tools/ep_owner_rank.py --expert -1 > $O/ep_ranks.jsonl 2> $O/ep_ranks.err || exit 1
timeout -k 10 600 bash tools/pmc_r06.sh ep_owner tools/ep_owner_rank.py > $O/pmc.log 2>&1 || exit 2
