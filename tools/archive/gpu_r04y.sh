#!/bin/bash
# C5 with each batch's rays in (expert, ray-midpoint Morton) order vs the stream's order
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04y; mkdir -p $O
for ord in none expert-mid; do
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$ord -o run -- python3 bench.py --workload c5 --no-cpu-baseline --c5-order $ord > $O/c5_$ord.json 2>$O/c5_$ord.err || exit 1
  find $O/prof_$ord -type f ! -name '*kernel_stats.csv' -delete
  python -c "import json; a=json.load(open('$O/c5_$ord.json')); r=a['roofline']; print('c5 $ord', a['value'], a['ms_per_step'], r['kernel_ms'], r.get('secondary',{}).get('kernel_ms'), r.get('secondary',{}).get('requests_over_distinct_segments'))"
  python - $O/prof_$ord <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if any(k in r["Name"] for k in ("hashgrid_fwd_pairs", "hashgrid_bwd_pairs", "adam_slots", "mlp_fwd_pairs", "mlp_bwd_dw_pairs")):
            print("   ", r["Name"][:70], r["Calls"], r["AverageNs"])
PY
done
