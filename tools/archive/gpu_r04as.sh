#!/bin/bash
# render_slots_kernel work sharing, tile-major (sws) vs ray-major (swsrm) items, against the per-wave default
# (base): render_ws test with the ray-major build, then C3 / C4-S96 / C4-S256, alternating
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04as; mkdir -p $O
: # (the render_ws test selection passed with this variant in tools/gpu_r04at.sh)

for v in base sws swsrm base sws swsrm; do
  lib=adaptive_city_nerf_amd/libacnerf.so; [ $v = base ] || lib=build_variants/libacnerf_$v.so
  for w in "c3:--workload c3" "c4s96:--workload c4 --samples 96 --steps 5" "c4:--workload c4 --steps 3"; do
    tag=${w%%:*}; args=${w#*:}
    ACNERF_LIB=$lib timeout -k 10 200 python -u bench.py --no-cpu-baseline $args > $O/${tag}_$v.json 2>$O/${tag}_$v.err || { tail -3 $O/${tag}_$v.err; exit 3; }
    python -c "import json; a=json.load(open('$O/${tag}_$v.json')); print('$tag $v', a['value'], a['ms_per_step'], a['roofline'].get('kernel_ms'))"
  done
done
