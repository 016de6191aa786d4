#!/bin/bash
# sweep rrLU pass grid size and deferred depth (bench.py, no extras)
for g in ${GRIDS:-256 512 1024 2048}; do
  for nb in ${NBS:-8}; do
    TCI_PASS_GRID=$g timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-extras --no-cpu --nb $nb > gpurun_out/sw_${g}_${nb}.log 2>&1 || exit 1
    python -c "import json;d=json.loads(open('gpurun_out/sw_${g}_${nb}.log').read().strip().splitlines()[-1]);r=d['roofline'];p=r['passes'];print('grid $g nb $nb', d['value'], d['ms_per_step'], 'ro', p['read_only_pass']['avg_ms'], 'wb', p['write_back_pass']['avg_ms'])"
  done
done
