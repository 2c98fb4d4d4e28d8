#!/bin/bash
# round 6: hash-grid forward through buffer loads (hashgrid_fwd_f2_buf) against the global-address gathers
# (ACN_HASH_FWD_BUF=0 variant): kernel / routed / training / meta parity tests, kernel A/B at the meta batch, meta and C5 step A/B (also hashgrid_fwd_pairs)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06w; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests/test_gpu_kernels.py tests/test_routed_glue.py tests/test_train.py tests/test_meta_gpu.py > $O/enc_tests.txt 2>&1 || exit 1
for rep in 1 2; do
  timeout -k 10 120 python -u tools/ab_hash_fwd.py > $O/hf_buf_$rep.jsonl 2> $O/hf_buf_$rep.err || exit 2
  ACNERF_LIB=build_variants/libacnerf_hfg.so timeout -k 10 120 python -u tools/ab_hash_fwd.py > $O/hf_glb_$rep.jsonl 2> $O/hf_glb_$rep.err || exit 2
  timeout -k 10 300 python -u bench.py --workload meta --no-cpu-baseline > $O/meta_buf_$rep.json 2> $O/meta_buf_$rep.err || exit 3
  ACNERF_LIB=build_variants/libacnerf_hfg.so timeout -k 10 300 python -u bench.py --workload meta --no-cpu-baseline > $O/meta_glb_$rep.json 2> $O/meta_glb_$rep.err || exit 3
  timeout -k 10 300 python -u bench.py --workload c5 --no-cpu-baseline > $O/c5_buf_$rep.json 2> $O/c5_buf_$rep.err || exit 4
  ACNERF_LIB=build_variants/libacnerf_hfg.so timeout -k 10 300 python -u bench.py --workload c5 --no-cpu-baseline > $O/c5_glb_$rep.json 2> $O/c5_glb_$rep.err || exit 4
done
