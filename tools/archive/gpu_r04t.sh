#!/bin/bash
# default build = render_slots_kernel again: its render tests; C4 (S = 96) counters of both routed kernels; meta lines
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04t; mkdir -p $O
RT=$PWD/build_variants/libacnerf_routed.so
timeout -k 10 600 python -u -m pytest tests/test_batch_independence.py tests/test_k8.py tests/test_gpu_kernels.py -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -le 1 ] || exit $rc
bash tools/pmc_r04.sh c4s --workload c4 --samples 96 --steps 2 --warmup 1 --no-cpu-baseline || exit 1
ACNERF_LIB=$RT bash tools/pmc_r04.sh c4r --workload c4 --samples 96 --steps 2 --warmup 1 --no-cpu-baseline || exit 2
python tools/pmc_fold_r04.py gpurun_out/pmc_c4r render_routed_kernel 61440000 $O/r04_pmc_c4s96_routed.json r04 "render_routed_kernel (C4, S = 96)" > $O/fold_c4r.txt
python tools/pmc_fold_r04.py gpurun_out/pmc_c4s render_slots_kernel 61440000 $O/r04_pmc_c4s96_slots.json r04 "render_slots_kernel (C4, S = 96)" > $O/fold_c4s.txt
cat $O/fold_c4r.txt $O/fold_c4s.txt
timeout -k 10 300 python -u bench.py --workload meta --no-cpu-baseline > $O/meta.json 2>$O/meta.err || exit 3
timeout -k 10 300 python -u bench.py --workload meta --mlp-precision amp --no-cpu-baseline > $O/meta_amp.json 2>$O/meta_amp.err || exit 4
for f in meta meta_amp; do
  python -c "import json; a=json.load(open('$O/$f.json')); r=a['roofline']; print('$f', a['value'], a['ms_per_step'], r.get('kernel_ms'), r.get('frac'), a.get('amp_scaler'))"
done
exit $rc
