#!/bin/bash
# A/B the rrLU bench under env settings: scripts/ab_env.sh "VAR=a VAR2=b" "VAR=c" ...
for cfg in "$@"; do
  tag=$(echo "$cfg" | tr " =/" "_+-")
  env $cfg timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-extras --no-cpu > gpurun_out/ab_${tag}.log 2>&1 || { tail -5 gpurun_out/ab_${tag}.log; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/ab_${tag}.log').read().strip().splitlines()[-1]);p=d['roofline']['passes'];print('$cfg', d['value'], d['ms_per_step'], 'ro', p['read_only_pass']['avg_ms'], 'wb', p['write_back_pass']['avg_ms'], p['read_only_pass'].get('avg_ms_by_pending_depth'))"
done
