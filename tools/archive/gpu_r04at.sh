#!/bin/bash
# re-run of the work-shared render test selection with the base library and with the slots-ws ray-major variant
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04at; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_render_ws.py -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "k4 or k8" > $O/base.log 2>&1; echo "base rc=$?"; tail -2 $O/base.log
ACNERF_LIB=build_variants/libacnerf_swsrm.so timeout -k 10 400 python -u -m pytest tests/test_render_ws.py -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "k4 or k8" > $O/swsrm.log 2>&1; echo "swsrm rc=$?"; grep -E "FAILED|passed|failed" $O/swsrm.log | tail -8
ACNERF_LIB=build_variants/libacnerf_sws.so timeout -k 10 400 python -u -m pytest tests/test_render_ws.py -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "k4 or k8" > $O/sws.log 2>&1; echo "sws rc=$?"; grep -E "FAILED|passed|failed" $O/sws.log | tail -8
exit 0
