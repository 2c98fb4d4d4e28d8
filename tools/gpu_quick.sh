#!/bin/bash
# tests selection + a few bench lines, each GPU step under its own limit, chained with &&
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
SEL=${1:-tests}
TAG=${2:-q}
shift 2
timeout -k 10 900 python -u -m pytest $SEL -m gpu -v --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_$TAG.log 2>&1
rc=$?
echo "pytest rc=$rc"
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for w in "$@"; do
  timeout -k 10 300 python -u bench.py $w > gpurun_out/bench_${TAG}_$(echo $w | tr -d ' -' ).json 2> gpurun_out/bench_${TAG}_$(echo $w | tr -d ' -').err || { echo "bench $w failed"; exit 3; }
done
echo "gpu_quick done"
