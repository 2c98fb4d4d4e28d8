#!/bin/bash
# round 6: XCD bands in ep_field_kernel -- EP correctness tests, every rank of the one-expert-per-GPU C4 layout with
# and without bands, counter passes of the busiest rank, the final render lines; LAST the forcezero self-check
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06q; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q -m gpu --timeout 600 --timeout-method thread tests/test_expert_parallel.py tests/test_rccl_world1.py > $O/ep_tests.txt 2>&1 || exit 1
timeout -k 10 300 python -u tools/ep_owner_rank.py --expert -1 > $O/ep_ranks_bands.jsonl 2> $O/ep_ranks_bands.err || exit 2
ACNERF_LIB=build_variants/libacnerf_nob.so timeout -k 10 300 python -u tools/ep_owner_rank.py --expert -1 > $O/ep_ranks_nob.jsonl 2> $O/ep_ranks_nob.err || exit 2
timeout -k 10 600 bash tools/pmc_r06.sh ep_owner tools/ep_owner_rank.py > $O/pmc_ep.log 2>&1 || exit 3
for rep in 1 2; do
  timeout -k 10 200 python -u bench.py --workload c2 --no-cpu-baseline > $O/c2_$rep.json 2> $O/c2_$rep.err || exit 5
  timeout -k 10 200 python -u bench.py --workload c3 --no-cpu-baseline > $O/c3_$rep.json 2> $O/c3_$rep.err || exit 5
  timeout -k 10 300 python -u bench.py --workload c4 --samples 96 --steps 5 --no-cpu-baseline > $O/c4s96_$rep.json 2> $O/c4s96_$rep.err || exit 5
done
ACNERF_LIB=build_variants/libacnerf_sc2fz.so timeout -k 10 400 python -u tools/dbg/selfcheck.py 30 > $O/sc_sc2fz.txt 2>&1 || exit 4
