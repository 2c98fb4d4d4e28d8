#!/bin/bash
# round-4 bench lines: hazard-pad cost (base vs nop0 / nop1 builds), C3 / C4-S96 routed render with cpu_baseline,
# C4 one-expert-per-GPU layout, C5 in fp16x3 and in use_amp, the float64 spread of the training gradients
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04n; mkdir -p $O
for v in base perf_nop0 perf_nop1; do
  if [ $v = base ]; then unset ACNERF_LIB; else export ACNERF_LIB=$PWD/build_variants/libacnerf_$v.so; fi
  timeout -k 10 150 python -u bench.py --no-cpu-baseline > $O/c2_$v.json 2>/dev/null || exit 3
  timeout -k 10 150 python -u bench.py --workload c3 --steps 100 --no-cpu-baseline > $O/c3_$v.json 2>/dev/null || exit 4
  python -c "import json; a=json.load(open('$O/c2_$v.json')); b=json.load(open('$O/c3_$v.json')); print('$v', 'c2', a['value'], a['roofline']['kernel_ms'], 'c3', b['value'], b['roofline']['kernel_ms'])"
done
unset ACNERF_LIB
timeout -k 10 200 python -u bench.py > $O/c2.json 2>$O/c2.err || exit 5
timeout -k 10 200 python -u bench.py --workload c3 > $O/c3.json 2>$O/c3.err || exit 6
timeout -k 10 300 python -u bench.py --workload c4 --samples 96 --steps 5 > $O/c4s96.json 2>$O/c4s96.err || exit 7
timeout -k 10 300 python -u bench.py --workload c4 --samples 96 --steps 5 --layout expert --no-cpu-baseline > $O/c4s96_expert.json 2>$O/c4e.err || exit 8
timeout -k 10 300 python -u bench.py --workload c5 > $O/c5.json 2>$O/c5.err || exit 9
timeout -k 10 300 python -u bench.py --workload c5 --mlp-precision amp --no-cpu-baseline > $O/c5_amp.json 2>$O/c5a.err || exit 10
for f in c2 c3 c4s96 c4s96_expert c5 c5_amp; do
  python -c "import json; a=json.load(open('$O/$f.json')); r=a['roofline']; print('$f', a['value'], a['ms_per_step'], r.get('kernel_ms'), r.get('frac'), r.get('traffic'), (a.get('cpu_baseline') or {}).get('value'))"
done
timeout -k 10 300 python -u tools/train_f64_spread.py --out $O/train_f64_spread.json 2>&1 | grep -v -i 'warning\|amdgpu.ids' | tail -30
