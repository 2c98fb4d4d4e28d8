#!/bin/bash
# round-4 final-build bench lines (after the work-shared render) (N = 1) with cpu_baseline, and the rocprof summary of the C2 headline
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04ar; mkdir -p $O
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c2 -o run -- python3 bench.py --steps 20 > $O/c2_prof.json 2>$O/c2_prof.err || exit 1
find $O/prof_c2 -type f ! -name '*kernel_stats.csv' -delete
timeout -k 10 200 python -u bench.py > $O/c2.json 2>$O/c2.err || exit 2
timeout -k 10 200 python -u bench.py --workload c3 > $O/c3.json 2>$O/c3.err || exit 3
timeout -k 10 300 python -u bench.py --workload c4 --samples 96 --steps 5 > $O/c4s96.json 2>$O/c4s96.err || exit 4
timeout -k 10 300 python -u bench.py --workload c4 --steps 3 > $O/c4.json 2>$O/c4.err || exit 5
timeout -k 10 300 python -u bench.py --workload c4 --samples 96 --steps 5 --layout expert --no-cpu-baseline > $O/c4s96_expert.json 2>$O/c4e.err || exit 6
timeout -k 10 300 python -u bench.py --workload c5 > $O/c5.json 2>$O/c5.err || exit 7
timeout -k 10 300 python -u bench.py --workload c5 --mlp-precision amp --no-cpu-baseline > $O/c5_amp.json 2>$O/c5a.err || exit 8
timeout -k 10 300 python -u bench.py --workload meta > $O/meta.json 2>$O/meta.err || exit 9
timeout -k 10 300 python -u bench.py --workload meta --mlp-precision amp --no-cpu-baseline > $O/meta_amp.json 2>$O/meta_amp.err || exit 10
for f in c2_prof c2 c3 c4s96 c4 c4s96_expert c5 c5_amp meta meta_amp; do
  python -c "import json; a=json.load(open('$O/$f.json')); r=a['roofline']; print('$f', a['value'], a['ms_per_step'], r.get('kernel_ms'), r.get('frac'), r.get('traffic'), (a.get('cpu_baseline') or {}).get('value'))"
done
