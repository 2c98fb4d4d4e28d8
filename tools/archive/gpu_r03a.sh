#!/bin/bash
# round 3, first GPU call: MLP-backward tests (ds_read_b64_tr_b16 transposed weight reads), the meta bench line
# with its new FLOP roofline, the gather-only ceiling microbenchmark, and rocprof summaries of both
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r03a
O=gpurun_out/r03a
timeout -k 10 600 python -u -m pytest tests/test_mlp_train_gpu.py tests/test_meta_gpu.py tests/test_train.py -m gpu -x -q \
  --timeout 240 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 300 python -u bench.py --workload meta --steps 10 --warmup 2 > $O/bench_meta.json 2> $O/bench_meta.err || { echo "bench meta failed"; tail $O/bench_meta.err; exit 3; }
cat $O/bench_meta.json
timeout -k 10 300 python -u tools/micro/hash_gather.py --out $O/hash_gather.json > $O/hash_gather.log 2>&1 || { echo "hash_gather failed"; tail $O/hash_gather.log; exit 4; }
tail -1 $O/hash_gather.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_meta -o run --output-format csv -- python3 bench.py --workload meta --steps 5 --warmup 1 --no-cpu-baseline > $O/prof_meta.log 2>&1 || { echo "rocprof meta failed"; exit 5; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_hg -o run --output-format csv -- python3 tools/micro/hash_gather.py --reps 20 --out $O/hash_gather_prof.json > $O/prof_hg.log 2>&1 || { echo "rocprof hg failed"; exit 6; }
echo "r03a done"
