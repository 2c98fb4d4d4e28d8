#!/bin/bash
# capture-keepalive workspaces, the replicated layout at world 2 on the HIP kernels, graph-capture suites
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04ab; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_graph_keepalive.py tests/test_parallel.py tests/test_train.py tests/test_meta_gpu.py tests/test_expert_parallel.py -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; tail -4 $O/pytest.log; exit $rc
