#!/bin/bash
# round 5: render_slots_kernel with 256-thread workgroups (288 VGPRs, one wave per SIMD) against the default 512
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05aj; mkdir -p $O
for v in default s256 default2 s256b; do
  case $v in s256*) export ACNERF_LIB=build_variants/libacnerf_s256.so;; *) unset ACNERF_LIB;; esac
  timeout -k 10 200 python -u bench.py --workload c3 --no-cpu-baseline > $O/c3_$v.json 2>$O/c3_$v.err || exit 1
  timeout -k 10 300 python -u bench.py --workload c4 --samples 96 --steps 5 --no-cpu-baseline > $O/c4s96_$v.json 2>$O/c4_$v.err || exit 2
  python -c "import json;a=json.load(open('$O/c3_$v.json'));b=json.load(open('$O/c4s96_$v.json'));print('$v c3', a['value'], 'c4s96', b['value'])"
done
