#!/bin/bash
# round 5 closing run on the final build: full GPU suite, smoke, and the render / C5 bench lines
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05fin2; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/suite.log 2>&1; rc=$?
tail -1 $O/suite.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 2
tail -1 $O/smoke.log
run() { tag=$1; shift; timeout -k 10 400 python -u bench.py "$@" > $O/$tag.json 2>$O/$tag.err || { echo "bench $tag failed"; tail -5 $O/$tag.err; exit 3; }
        python -c "import json;d=json.load(open('$O/$tag.json'));print('$tag', d['value'], d['ms_per_step'], d['roofline']['frac'])"; }
run c2
run c3 --workload c3
run c4s96 --workload c4 --samples 96 --steps 5
run c4 --workload c4 --steps 3 --no-cpu-baseline
run c5 --workload c5
