#!/bin/bash
# round 6: SLP vectorizer cost thresholds on render.hip (spill-free at 5 and -3) against the no-SLP default
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06s; mkdir -p $O
for rep in 1 2; do
for v in default slp5 slpm3 slp0; do
  if [ $v = default ]; then unset ACNERF_LIB; else export ACNERF_LIB=build_variants/libacnerf_$v.so; fi
  timeout -k 10 200 python -u bench.py --workload c2 --no-cpu-baseline > $O/c2_${v}_$rep.json 2> $O/c2_${v}_$rep.err || exit 2
  timeout -k 10 200 python -u bench.py --workload c3 --no-cpu-baseline > $O/c3_${v}_$rep.json 2> $O/c3_${v}_$rep.err || exit 3
  timeout -k 10 300 python -u bench.py --workload c4 --samples 96 --steps 5 --no-cpu-baseline > $O/c4s96_${v}_$rep.json 2> $O/c4s96_${v}_$rep.err || exit 4
done
done
unset ACNERF_LIB
for b in 32 8; do
  timeout -k 10 300 python -u tools/ep_owner_rank.py --order depth-tiled --block $b > $O/ep_depth_b$b.jsonl 2> $O/ep_depth_b$b.err || exit 5
done
timeout -k 10 300 python -u tools/ep_owner_rank.py > $O/ep_sample.jsonl 2> $O/ep_sample.err || exit 5
