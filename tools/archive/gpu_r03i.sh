#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest tests/test_k8.py -m gpu -q -k "split or k8_vs_reference" --timeout 120 --timeout-method thread -p no:cacheprovider 2>&1 | tail -2
bash tools/gpu_prof.sh c3s "--workload c3 --steps 50" && bash tools/gpu_prof.sh c4s96 "--workload c4 --samples 96 --steps 5"
