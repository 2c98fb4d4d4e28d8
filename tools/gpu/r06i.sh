#!/bin/bash
# round 6: the buffer-load hash gathers (ACN_XPAIR=2) -- production-layout hash self-check, and C2 / C3 / C4-S96 A/B
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06i; mkdir -p $O
ACNERF_LIB=build_variants/libacnerf_fcxp2.so timeout -k 10 300 python -u tools/dbg/selfcheck.py 40 > $O/sc_fcxp2.txt 2>&1 || exit 1
for rep in 1 2; do
for v in default xp2; do
  if [ $v = xp2 ]; then export ACNERF_LIB=build_variants/libacnerf_xp2.so; else unset ACNERF_LIB; fi
  timeout -k 10 200 python -u bench.py --workload c2 --no-cpu-baseline > $O/c2_${v}_$rep.json 2> $O/c2_${v}_$rep.err || exit 2
  timeout -k 10 200 python -u bench.py --workload c3 --no-cpu-baseline > $O/c3_${v}_$rep.json 2> $O/c3_${v}_$rep.err || exit 3
  timeout -k 10 300 python -u bench.py --workload c4 --samples 96 --steps 5 --no-cpu-baseline > $O/c4s96_${v}_$rep.json 2> $O/c4s96_${v}_$rep.err || exit 4
done
done
