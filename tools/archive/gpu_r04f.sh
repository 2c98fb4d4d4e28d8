#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 200 python -u tools/dbg/rt_det2.py 2>&1 | grep -v -i 'warning\|amdgpu.ids'
