#!/bin/bash
# round 6: hash levels in flight (ACN_HASH_DEPTH 1 / 2 / 3) and per-corner buffer gathers (ACN_XPAIR=3) on the
# depth-tiled renders: C2 / C3 / C4-S96 A/B
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06ag; mkdir -p $O
for rep in 1 2; do
  for v in default hd3 hd1 xp3; do
    if [ $v = default ]; then unset ACNERF_LIB; else export ACNERF_LIB=build_variants/libacnerf_$v.so; fi
    timeout -k 10 200 python -u bench.py --workload c2 --no-cpu-baseline > $O/c2_${v}_$rep.json 2> $O/c2_${v}_$rep.err || exit 2
    timeout -k 10 200 python -u bench.py --workload c3 --no-cpu-baseline > $O/c3_${v}_$rep.json 2> $O/c3_${v}_$rep.err || exit 3
    timeout -k 10 300 python -u bench.py --workload c4 --samples 96 --steps 5 --no-cpu-baseline > $O/c4s96_${v}_$rep.json 2> $O/c4s96_${v}_$rep.err || exit 4
  done
done
unset ACNERF_LIB
