#!/bin/bash
# round 6: buffer-load hash gathers (XPAIR 3, with and without the SLP vectorizer): hash self-check in the sensitive
# and the production layouts, then C2 / C3 / C4-S96 against the round-5 build (global-address gathers) and XPAIR 2
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06j; mkdir -p $O
ACNERF_LIB=build_variants/libacnerf_sc2fcb3ns.so timeout -k 10 300 python -u tools/dbg/selfcheck.py 20 > $O/sc_sc2fcb3ns.txt 2>&1 || exit 1
ACNERF_LIB=build_variants/libacnerf_fcb3ns.so timeout -k 10 300 python -u tools/dbg/selfcheck.py 40 > $O/sc_fcb3ns.txt 2>&1 || exit 1
for rep in 1 2; do
for v in g0 xp2 b3 b3ns; do
  export ACNERF_LIB=build_variants/libacnerf_$v.so
  timeout -k 10 200 python -u bench.py --workload c2 --no-cpu-baseline > $O/c2_${v}_$rep.json 2> $O/c2_${v}_$rep.err || exit 2
  timeout -k 10 200 python -u bench.py --workload c3 --no-cpu-baseline > $O/c3_${v}_$rep.json 2> $O/c3_${v}_$rep.err || exit 3
  timeout -k 10 300 python -u bench.py --workload c4 --samples 96 --steps 5 --no-cpu-baseline > $O/c4s96_${v}_$rep.json 2> $O/c4s96_${v}_$rep.err || exit 4
done
done
