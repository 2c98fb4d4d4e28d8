#!/bin/bash
# round 5: G rounds of render_slots_kernel per slot choice (one barrier per group): parity, then C3 / C4 A/B
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05am; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_render_ws.py tests/test_k8.py tests/test_batch_independence.py tests/test_determinism_gpu.py tests/test_gpu_kernels.py tests/test_parallel.py -q -m gpu -x --timeout 300 --timeout-method thread > $O/parity.log 2>&1 || { tail -30 $O/parity.log; exit 1; }
tail -1 $O/parity.log
for v in g4 g1 g2 g4b g1b; do
  case $v in g4*) unset ACNERF_LIB;; g1*) export ACNERF_LIB=build_variants/libacnerf_g1.so;; g2*) export ACNERF_LIB=build_variants/libacnerf_g2.so;; esac
  timeout -k 10 200 python -u bench.py --workload c3 --no-cpu-baseline > $O/c3_$v.json 2>$O/c3_$v.err || exit 2
  timeout -k 10 300 python -u bench.py --workload c4 --samples 96 --steps 5 --no-cpu-baseline > $O/c4s96_$v.json 2>$O/c4s96_$v.err || exit 3
  timeout -k 10 300 python -u bench.py --workload c4 --steps 3 --no-cpu-baseline > $O/c4_$v.json 2>$O/c4_$v.err || exit 4
  python -c "import json;a=json.load(open('$O/c3_$v.json'));b=json.load(open('$O/c4s96_$v.json'));c=json.load(open('$O/c4_$v.json'));print('$v c3', a['value'], 'c4s96', b['value'], 'c4', c['value'])"
done
