#!/bin/bash
# round 6: (1) hash-feature detector on the final build's layout (x-paired buffer gathers, fence off, no SLP);
# (2) one rank of the one-expert-per-GPU C4 layout: every rank timed, kernel trace + counter passes of the busiest;
# (3) LAST: the 512-thread slots self-check build with every s_waitcnt forced to zero (round 5 faulted there)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06o; mkdir -p $O
ACNERF_LIB=build_variants/libacnerf_fcfinal.so timeout -k 10 300 python -u tools/dbg/selfcheck.py 40 > $O/sc_fcfinal.txt 2>&1 || exit 1
ACNERF_LIB=build_variants/libacnerf_sc2fcfinal.so timeout -k 10 300 python -u tools/dbg/selfcheck.py 20 > $O/sc_sc2fcfinal.txt 2>&1 || exit 1
timeout -k 10 300 python -u tools/ep_owner_rank.py --expert -1 > $O/ep_ranks.jsonl 2> $O/ep_ranks.err || exit 2
timeout -k 10 600 bash tools/pmc_r06.sh ep_owner tools/ep_owner_rank.py > $O/pmc_ep.log 2>&1 || exit 3
for rep in 1 2; do
for v in default pk; do
  if [ $v = default ]; then unset ACNERF_LIB; else export ACNERF_LIB=build_variants/libacnerf_$v.so; fi
  timeout -k 10 200 python -u bench.py --workload c2 --no-cpu-baseline > $O/c2_${v}_$rep.json 2> $O/c2_${v}_$rep.err || exit 5
  timeout -k 10 200 python -u bench.py --workload c3 --no-cpu-baseline > $O/c3_${v}_$rep.json 2> $O/c3_${v}_$rep.err || exit 5
  timeout -k 10 300 python -u bench.py --workload c4 --samples 96 --steps 5 --no-cpu-baseline > $O/c4s96_${v}_$rep.json 2> $O/c4s96_${v}_$rep.err || exit 5
done
done
unset ACNERF_LIB
ACNERF_LIB=build_variants/libacnerf_sc2fz.so timeout -k 10 400 python -u tools/dbg/selfcheck.py 30 > $O/sc_sc2fz.txt 2>&1 || exit 4
