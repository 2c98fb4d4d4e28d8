#!/bin/bash
# round 5: is the field kernel's one-off a run-to-run difference?  field_fwd repeated on the current build and on
# the round-4 build; then the failing test alone, several times
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05b; mkdir -p $O
timeout -k 10 300 python -u tools/dbg/field_repeat.py 200 > $O/field_repeat_cur.txt 2>&1 || exit 1
ACNERF_LIB=build_variants/libacnerf_r04.so timeout -k 10 300 python -u tools/dbg/field_repeat.py 200 > $O/field_repeat_r04.txt 2>&1 || exit 2
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "field_vs_reference" > $O/field_test.log 2>&1 || exit 3
timeout -k 10 600 python -u -m pytest tests/test_expert_parallel.py -x -q -m gpu --timeout 300 --timeout-method thread > $O/ep_tests.log 2>&1 || exit 4
