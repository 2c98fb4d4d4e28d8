#!/bin/bash
# round 5: XCD bands in render_slots_kernel for the expert-sorted C3 batch (each XCD's L2 sees ~one expert)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05t; mkdir -p $O
for v in default band default2 band2; do
  case $v in band*) export ACNERF_LIB=build_variants/libacnerf_band.so;; *) unset ACNERF_LIB;; esac
  timeout -k 10 200 python -u bench.py --workload c3 --no-cpu-baseline > $O/c3_$v.json 2>$O/c3_$v.err || exit 1
  python -c "import json;d=json.load(open('$O/c3_$v.json'));print('c3 $v', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])"
done
for v in default band; do
  case $v in band*) export ACNERF_LIB=build_variants/libacnerf_band.so;; *) unset ACNERF_LIB;; esac
  timeout -k 10 300 python -u bench.py --workload c4 --samples 96 --steps 5 --no-cpu-baseline > $O/c4s96_$v.json 2>$O/c4_$v.err || exit 2
  python -c "import json;d=json.load(open('$O/c4s96_$v.json'));print('c4s96 $v', d['value'], d['ms_per_step'])"
done
