#!/bin/bash
# round 5: the expert-phase routed work-shared render: parity suites, C3 / C4 against the slots kernel, RCCL test
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05q; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_render_ws.py tests/test_k8.py tests/test_batch_independence.py tests/test_determinism_gpu.py tests/test_gpu_kernels.py -q -m gpu -x --timeout 300 --timeout-method thread > $O/parity.log 2>&1 || exit 1
timeout -k 10 200 python -u bench.py --workload c3 --no-cpu-baseline > $O/c3_rws.json 2>$O/c3_rws.err || exit 2
ACNERF_LIB=build_variants/libacnerf_slots.so timeout -k 10 200 python -u bench.py --workload c3 --no-cpu-baseline > $O/c3_slots.json 2>$O/c3_slots.err || exit 3
timeout -k 10 300 python -u bench.py --workload c4 --samples 96 --steps 5 --no-cpu-baseline > $O/c4s96_rws.json 2>$O/c4_rws.err || exit 4
ACNERF_LIB=build_variants/libacnerf_slots.so timeout -k 10 300 python -u bench.py --workload c4 --samples 96 --steps 5 --no-cpu-baseline > $O/c4s96_slots.json 2>$O/c4_slots.err || exit 5
timeout -k 10 300 python -u bench.py --workload c4 --steps 3 --no-cpu-baseline > $O/c4_rws.json 2>$O/c4b_rws.err || exit 6
timeout -k 10 400 python -u -m pytest tests/test_rccl_world1.py -v -s -m gpu --timeout 380 --timeout-method thread > $O/rccl.log 2>&1
timeout -k 10 600 python -u -m pytest tests/test_amp.py tests/test_expert_parallel.py -q -m gpu --timeout 300 --timeout-method thread > $O/tests.log 2>&1
