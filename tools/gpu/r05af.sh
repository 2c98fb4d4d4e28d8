#!/bin/bash
# round 5: the planned exchange's live-byte statistic computed from the routed device counts (not the split sizes)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05af; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_expert_parallel.py -q -m gpu -x --timeout 300 --timeout-method thread > $O/ep.log 2>&1 || { tail -30 $O/ep.log; exit 1; }
tail -1 $O/ep.log
timeout -k 10 300 python -u bench.py --workload c4 --samples 96 --layout expert --steps 3 --no-cpu-baseline > $O/c4s96_expert.json 2>$O/c4e.err || exit 2
python -c "import json;d=json.load(open('$O/c4s96_expert.json'));print(d['value'], d['ms_per_step'], d['exchange'])"
