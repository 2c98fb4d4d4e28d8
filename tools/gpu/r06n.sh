#!/bin/bash
# round 6: the final-candidate build (buffer-load hash gathers, operand fence compiled out, render.hip without SLP):
# full GPU suite + smoke, then A/B against the fenced render / training MLP (C2, C3, C4-S96, meta)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06n; mkdir -p $O
unset ACNERF_LIB
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_suite.txt 2>&1 || exit 1
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || exit 2
for rep in 1 2; do
for v in default fon; do
  if [ $v = default ]; then unset ACNERF_LIB; else export ACNERF_LIB=build_variants/libacnerf_$v.so; fi
  timeout -k 10 200 python -u bench.py --workload c2 --no-cpu-baseline > $O/c2_${v}_$rep.json 2> $O/c2_${v}_$rep.err || exit 3
  timeout -k 10 200 python -u bench.py --workload c3 --no-cpu-baseline > $O/c3_${v}_$rep.json 2> $O/c3_${v}_$rep.err || exit 3
  timeout -k 10 300 python -u bench.py --workload c4 --samples 96 --steps 5 --no-cpu-baseline > $O/c4s96_${v}_$rep.json 2> $O/c4s96_${v}_$rep.err || exit 3
done
unset ACNERF_LIB
timeout -k 10 300 python -u bench.py --workload meta --no-cpu-baseline > $O/meta_default_$rep.json 2> $O/meta_default_$rep.err || exit 4
ACNERF_LIB=build_variants/libacnerf_mlpfon.so timeout -k 10 300 python -u bench.py --workload meta --no-cpu-baseline > $O/meta_fon_$rep.json 2> $O/meta_fon_$rep.err || exit 4
done
