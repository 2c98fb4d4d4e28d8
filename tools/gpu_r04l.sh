#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
for v in nop1 nop3; do
  export ACNERF_LIB=$PWD/build_variants/libacnerf_$v.so
  echo "== $v"; timeout -k 10 200 python -u tools/dbg/rt_check.py 2>&1 | grep -v -i 'warning\|amdgpu.ids'
done
for v in base perf_nop1 perf_nop2; do
  if [ $v = base ]; then unset ACNERF_LIB; else export ACNERF_LIB=$PWD/build_variants/libacnerf_$v.so; fi
  timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/r04l_c2_$v.json 2>/dev/null || exit 3
  timeout -k 10 200 python -u bench.py --workload c3 --steps 100 --no-cpu-baseline > gpurun_out/r04l_c3_$v.json 2>/dev/null || exit 4
  python -c "import json; a=json.load(open('gpurun_out/r04l_c2_$v.json')); b=json.load(open('gpurun_out/r04l_c3_$v.json')); print('$v', 'c2', a['value'], a['roofline']['kernel_ms'], 'c3', b['value'], b['roofline']['kernel_ms'])"
done
unset ACNERF_LIB
timeout -k 10 400 python -u tools/train_f64_spread.py --out gpurun_out/train_f64_spread.json 2>&1 | grep -v -i 'warning\|amdgpu.ids' | tail -40
