#!/bin/bash
# round 6: VMEM address WAR probe; the RCCL world-1 test with graph release + a real destroy_process_group
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06d; mkdir -p $O
timeout -k 10 300 tools/micro/vmem_war_probe 4096 100 > $O/vmem_war.txt 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 880 --timeout-method thread tests/test_rccl_world1.py > $O/rccl_world1.txt 2>&1 || exit 2
