#!/bin/bash
# tests of this round's changes (AMP incl. meta, EP renderer, segment-mapped Adam), then the C5 Adam A/B
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04q; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_amp.py tests/test_expert_parallel.py tests/test_train.py -m gpu -v -rP --timeout 200 --timeout-method thread -p no:cacheprovider -k "amp or renderer or segment or adam or world1 or world2 or bounded" > $O/pytest.log 2>&1
rc=$?; grep -E "passed|failed|FAILED|ERROR|AMPREPORT" $O/pytest.log | tail -24
echo "tests rc=$rc"
[ $rc -le 1 ] || exit $rc
bash tools/ab_c5.sh $O/ab_c5.txt base seglds0 base seglds0 || exit 2
