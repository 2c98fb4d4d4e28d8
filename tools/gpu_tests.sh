#!/bin/bash
# GPU test pass: the given test selection (default: whole -m gpu suite), no -x so every failure shows.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
SEL=${1:-tests}
TAG=${2:-t}
timeout -k 10 1000 python -u -m pytest $SEL -m gpu -v --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_$TAG.log 2>&1
echo "gpu_tests exit=$?"
