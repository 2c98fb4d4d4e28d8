#!/bin/bash
# round 6: x-paired buffer gathers without the SLP vectorizer (x2ns) against per-corner buffer gathers (b3ns)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06k; mkdir -p $O
for rep in 1 2; do
for v in x2ns b3ns xp2; do
  export ACNERF_LIB=build_variants/libacnerf_$v.so
  timeout -k 10 200 python -u bench.py --workload c2 --no-cpu-baseline > $O/c2_${v}_$rep.json 2> $O/c2_${v}_$rep.err || exit 2
  timeout -k 10 200 python -u bench.py --workload c3 --no-cpu-baseline > $O/c3_${v}_$rep.json 2> $O/c3_${v}_$rep.err || exit 3
  timeout -k 10 300 python -u bench.py --workload c4 --samples 96 --steps 5 --no-cpu-baseline > $O/c4s96_${v}_$rep.json 2> $O/c4s96_${v}_$rep.err || exit 4
done
done
