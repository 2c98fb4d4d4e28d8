#!/bin/bash
# split Adam (early pass on a side stream) + the AMP fp16 dW stage: training tests, then C5 / meta lines
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04u; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_train.py tests/test_amp.py tests/test_meta_gpu.py tests/test_mlp_train_gpu.py -m gpu -v -rP --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; grep -E "passed|failed|FAILED|ERROR|AMPREPORT" $O/pytest.log | tail -24; echo "tests rc=$rc"
[ $rc -le 1 ] || exit $rc
for e in 1 0 1 0; do
  ACN_ADAM_EARLY=$e timeout -k 10 200 python -u bench.py --workload c5 --no-cpu-baseline > $O/c5_early$e.json 2>$O/c5_early$e.err || exit 3
  python -c "import json; a=json.load(open('$O/c5_early$e.json')); r=a['roofline']; print('c5 early=$e', a['value'], a['ms_per_step'], r['kernel_ms'], r['frac'], a['val_psnr_db']['after'])"
done
timeout -k 10 300 python -u bench.py --workload meta --mlp-precision amp --no-cpu-baseline > $O/meta_amp.json 2>$O/meta_amp.err || exit 4
timeout -k 10 300 python -u bench.py --workload meta --no-cpu-baseline > $O/meta.json 2>$O/meta.err || exit 5
for f in meta meta_amp; do
  python -c "import json; a=json.load(open('$O/$f.json')); r=a['roofline']; print('$f', a['value'], a['ms_per_step'], r.get('kernel_ms'), r.get('frac'), a.get('amp_scaler'))"
done
exit $rc
