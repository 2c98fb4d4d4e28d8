#!/bin/bash
# segment-mapped Adam with the map bytes loaded one iteration ahead (ACN_ADAM_MAP_PIPE): Adam / training tests,
# then the C5 A/B against the previous loop (pipe0), alternating
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04ah; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_train.py tests/test_amp.py -m gpu -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "segment or adam or amp or skip" > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; echo "tests rc=$rc"
[ $rc -eq 0 ] || exit $rc
bash tools/ab_c5.sh $O/ab_c5.txt base pipe0 base pipe0 || exit 2
