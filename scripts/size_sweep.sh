#!/bin/bash
# rrLU pass time vs matrix size (fixed per-pass overhead vs streamed bytes):
#   scripts/size_sweep.sh "4096 4096" "8192 8192" ...
for mn in "$@"; do
  set -- $mn
  tag="${1}x${2}"
  timeout -k 10 300 python bench.py --m $1 --n $2 --steps 3 --warmup 1 --no-extras --no-cpu > gpurun_out/sz_${tag}.log 2>&1 || { tail -5 gpurun_out/sz_${tag}.log; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/sz_${tag}.log').read().strip().splitlines()[-1]);p=d['roofline']['passes'];print('$tag', d['value'], d['ms_per_step'], 'ro', p['read_only_pass']['avg_ms'], p['read_only_pass']['GBps'], 'wb', p['write_back_pass']['avg_ms'], 'stream', d['roofline']['measured_stream_read_GBps'])"
done
