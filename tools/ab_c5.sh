#!/bin/bash
# A/B build_variants/*.so on the C5 routed-adaptation bench (Adam + hash-backward kernel times).
# Usage (on the GPU box): tools/ab_c5.sh OUTFILE name1 name2 ...   ("base" = the regular build)
set -o pipefail
OUT=$1; shift
mkdir -p gpurun_out
: > $OUT
for v in "$@"; do
  lib=adaptive_city_nerf_amd/libacnerf.so
  [ "$v" = base ] || lib=build_variants/libacnerf_$v.so
  ACNERF_LIB=$lib timeout -k 10 200 python bench.py --workload c5 --steps 30 --warmup 5 --no-cpu-baseline \
      > gpurun_out/abc5_$v.json 2> gpurun_out/abc5_$v.err || { echo "variant $v failed"; exit 1; }
  python - "$v" >> $OUT <<'PY'
import json, sys
v = sys.argv[1]
d = json.loads(open(f"gpurun_out/abc5_{v}.json").read().strip().splitlines()[-1])
r = d["roofline"]
print(f"{v:8s} ms/step={d['ms_per_step']:.4f} adam_ms={r['kernel_ms']:.4f} frac={r['frac']:.3f} "
      f"hash_bwd_ms={r.get('secondary', {}).get('kernel_ms')} psnr_after={d['val_psnr_db']['after']}")
PY
done
cat $OUT
