#!/bin/bash
# round-4 kernel statistics of the meta-training step (fp32-accurate and use_amp)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04ap; mkdir -p $O
for m in fp16x3 amp; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$m -o run -- python3 bench.py --workload meta --mlp-precision $m --steps 5 --warmup 2 --no-cpu-baseline > $O/meta_$m.json 2>$O/meta_$m.err || { tail -3 $O/meta_$m.err; exit 2; }
  f=$(find $O/prof_$m -name '*kernel_stats.csv' | head -1); cp $f $O/meta_${m}_kernel_stats.csv
  find $O/prof_$m -type f ! -name '*kernel_stats.csv' -delete
  python -c "import json; a=json.loads(open('$O/meta_$m.json').read().strip().splitlines()[-1]); print('meta $m', a['value'], a['ms_per_step'])"
done
