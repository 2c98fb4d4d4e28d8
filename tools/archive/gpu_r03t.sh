#!/bin/bash
# per-step kernel counts of the C5 graph replay: kernel stats at 20 and 60 timed steps, differenced
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03t
mkdir -p $O
for n in 20 60; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p$n -o run -- python3 bench.py --workload c5 --steps $n --no-cpu-baseline > $O/p$n.log 2>&1 || { echo "prof $n failed"; exit 4; }
  find $O/p$n -type f ! -name '*kernel_stats.csv' -delete
done
python3 - <<'PY'
import csv
a={r['Name']:(int(r['Calls']),float(r['TotalDurationNs'])) for r in csv.DictReader(open('gpurun_out/r03t/p20/run_kernel_stats.csv'))}
b={r['Name']:(int(r['Calls']),float(r['TotalDurationNs'])) for r in csv.DictReader(open('gpurun_out/r03t/p60/run_kernel_stats.csv'))}
rows=[]
for k,(c,t) in b.items():
    c0,t0=a.get(k,(0,0.0))
    if c-c0>0: rows.append(((t-t0)/40/1e3,(c-c0)/40,k[:90]))
rows.sort(reverse=True)
tot=sum(r[0] for r in rows)
print(f"per-step GPU time {tot:.1f} us")
for t,c,k in rows[:40]: print(f"{t:8.1f} us  {c:5.2f}/step  {k}")
PY
