#!/bin/bash
# round 5: ray_expert_mask without the per-expert quotients (2K square roots per sample instead of 3K + 3K
# divisions): render parity suites, C3 / C4 lines, section profile
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05ak; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_render_ws.py tests/test_k8.py tests/test_batch_independence.py tests/test_determinism_gpu.py tests/test_gpu_kernels.py tests/test_parallel.py tests/test_expert_parallel.py tests/test_train.py tests/test_routed_glue.py tests/test_amp.py tests/test_occ_gpu.py tests/test_data_gpu.py -q -m gpu -x --timeout 300 --timeout-method thread > $O/parity.log 2>&1 || { tail -30 $O/parity.log; exit 1; }
tail -1 $O/parity.log
run() { tag=$1; shift; timeout -k 10 300 python -u bench.py "$@" > $O/$tag.json 2>$O/$tag.err || { echo "bench $tag failed"; tail -5 $O/$tag.err; exit 2; }
        python -c "import json;d=json.load(open('$O/$tag.json'));print('$tag', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])"; }
run c3 --workload c3 --no-cpu-baseline
run c4s96 --workload c4 --samples 96 --steps 5 --no-cpu-baseline
run c4 --workload c4 --steps 3 --no-cpu-baseline
ACNERF_LIB=build_variants/libacnerf_slprof.so timeout -k 10 300 python -u tools/dbg/slots_prof.py > $O/slprof.txt 2>&1 || exit 3
cat $O/slprof.txt
timeout -k 10 240 python -u bench.py --workload c5 --steps 30 --warmup 5 --no-cpu-baseline > $O/c5.json 2>$O/c5.err || exit 4
python -c "import json;d=json.load(open('$O/c5.json'));print('c5', d['ms_per_step'], d['roofline']['kernel_ms'])"
