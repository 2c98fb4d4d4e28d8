#!/bin/bash
# closing C2 confirmation on a fresh box: the default bench line (with the CPU baseline) twice, and C5 once
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04ax; mkdir -p $O
for i in 1 2; do
  timeout -k 10 300 python -u bench.py > $O/c2_$i.json 2>$O/c2_$i.err || { tail -3 $O/c2_$i.err; exit 1; }
  python -c "import json; a=json.load(open('$O/c2_$i.json')); print('c2', a['value'], a['ms_per_step'], a['roofline']['kernel_ms'], a['roofline']['frac'], a['cpu_baseline']['value'])"
done
timeout -k 10 300 python -u bench.py --workload c5 > $O/c5.json 2>$O/c5.err || { tail -3 $O/c5.err; exit 2; }
python -c "import json; a=json.load(open('$O/c5.json')); r=a['roofline']; print('c5', a['value'], a['ms_per_step'], r['kernel_ms'], r['secondary']['kernel_ms'], (a.get('cpu_baseline') or {}).get('value'))"
