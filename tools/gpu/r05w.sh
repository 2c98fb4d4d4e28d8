#!/bin/bash
# round 5 final build: the meta-training lines and their rocprof summary
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05w; mkdir -p $O
run() { tag=$1; shift; timeout -k 10 500 python -u bench.py "$@" > $O/$tag.json 2>$O/$tag.err || { echo "bench $tag failed"; tail -5 $O/$tag.err; exit 1; }
        python -c "import json;d=json.load(open('$O/$tag.json'));print('$tag', d['value'], d['ms_per_step'], d['roofline']['frac'])"; }
run meta --workload meta
run meta_amp --workload meta --mlp-precision amp --no-cpu-baseline
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c5 -o run -- python3 bench.py --workload c5 --no-cpu-baseline > $O/prof_c5.log 2>&1 || exit 2
find $O/prof_c5 -type f ! -name '*kernel_stats.csv' -delete
