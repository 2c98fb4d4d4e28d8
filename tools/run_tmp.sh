set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_train.py tests/test_hash_det.py -m gpu -q --timeout 240 --timeout-method thread -k "hash or adapt or routed or det" > gpurun_out/pt_merge.log 2>&1
echo pytest rc=$?
for v in base nomerge m3 m8; do
  lib=adaptive_city_nerf_amd/libacnerf.so; [ $v = base ] || lib=build_variants/libacnerf_$v.so
  ACNERF_LIB=$lib timeout -k 10 120 python -u tools/hash_det_time.py > gpurun_out/hdt_$v.txt 2>&1 || exit 1
done
bash tools/ab_c5.sh gpurun_out/ab_merge.txt base nomerge m3 m8 base
