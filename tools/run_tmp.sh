set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
ACN_TRACE_MARK=1 timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tr_meta2 -o run -- python3 bench.py --workload meta --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/tr_meta2.log 2>&1 &&
python tools/trace_busy.py gpurun_out/tr_meta2 5 30
