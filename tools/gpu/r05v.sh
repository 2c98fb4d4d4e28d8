#!/bin/bash
# round 5 final build: the bench lines (C2 with its rocprof summary, C3, C4, C5, meta) and their CPU baselines
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05v; mkdir -p $O
run() { tag=$1; shift; timeout -k 10 400 python -u bench.py "$@" > $O/$tag.json 2>$O/$tag.err || { echo "bench $tag failed"; tail -5 $O/$tag.err; exit 1; }
        python -c "import json;d=json.load(open('$O/$tag.json'));print('$tag', d['value'], d['ms_per_step'], d['roofline']['frac'])"; }
run c2 --steps 20
run c2_200
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c2 -o run -- python3 bench.py --steps 20 --no-cpu-baseline > $O/prof_c2.log 2>&1 || exit 2
find $O/prof_c2 -type f ! -name '*kernel_stats.csv' -delete
run c3 --workload c3
run c4s96 --workload c4 --samples 96 --steps 5
run c4 --workload c4 --steps 3 --no-cpu-baseline
run c4s96_expert --workload c4 --samples 96 --layout expert --steps 3 --no-cpu-baseline
run c5 --workload c5
run c5_amp --workload c5 --mlp-precision amp --no-cpu-baseline
