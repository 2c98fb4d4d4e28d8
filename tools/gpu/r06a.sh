#!/bin/bash
# round 6: trans-forwarding probe + the slots self-check baseline of this session's build
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06a; mkdir -p $O
timeout -k 10 300 tools/micro/trans_probe 2048 100 > $O/trans_probe.txt 2>&1 || exit 1
ACNERF_LIB=build_variants/libacnerf_sc2.so timeout -k 10 400 python -u tools/dbg/selfcheck.py 30 > $O/sc_sc2.txt 2>&1 || exit 2
