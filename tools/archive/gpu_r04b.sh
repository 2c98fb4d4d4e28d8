#!/bin/bash
# round 4 call b: stable ray order + batch-independence tests; C3/C4 A/B (XCD bands, shared table)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04b
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_batch_independence.py tests/test_gpu_kernels.py tests/test_k8.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; grep -E "passed|failed|FAILED|ERROR" $O/pytest.log | tail -15; [ $rc -eq 0 ] || exit $rc
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c2 -o run -- python3 bench.py --steps 50 --no-cpu-baseline > $O/prof_c2.log 2>&1 || { echo "prof c2 failed"; exit 3; }
find $O/prof_c2 -type f ! -name '*kernel_stats.csv' -delete
for v in base band; do
  if [ $v = band ]; then export ACNERF_LIB=$PWD/build_variants/libacnerf_band.so; else unset ACNERF_LIB; fi
  timeout -k 10 200 python -u bench.py --workload c3 --steps 100 --no-cpu-baseline > $O/c3_$v.json 2>>$O/err.log || exit 4
  timeout -k 10 200 python -u bench.py --workload c4 --samples 96 --steps 3 --no-cpu-baseline > $O/c4s96_$v.json 2>>$O/err.log || exit 5
done
unset ACNERF_LIB
timeout -k 10 200 python -u bench.py --workload c3 --steps 100 --no-cpu-baseline --diag-shared-table > $O/c3_shared.json 2>>$O/err.log || exit 6
timeout -k 10 200 python -u bench.py --workload c4 --samples 96 --steps 3 --no-cpu-baseline --diag-shared-table > $O/c4s96_shared.json 2>>$O/err.log || exit 7
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c3 -o run -- python3 bench.py --workload c3 --steps 50 --no-cpu-baseline > $O/prof_c3.log 2>&1 || { echo "prof c3 failed"; exit 8; }
find $O/prof_c3 -type f ! -name '*kernel_stats.csv' -delete
for f in $O/*.json; do python -c "import json,sys; d=json.load(open('$f')); print('$f', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])"; done
echo "r04b done"
