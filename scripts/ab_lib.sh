#!/bin/bash
# A/B the rrLU bench over library variants x env settings:
#   LIBS="default noxs" scripts/ab_lib.sh "VAR=a" "VAR=b" ...   (variants from `make variant NAME=...`)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
for lib in ${LIBS:-default}; do
  for cfg in "$@"; do
    if [ "$lib" = default ]; then unset TCI_HIP_LIB; else export TCI_HIP_LIB="$R/tensorcrossinterpolation.jl_amd/lib/variants/$lib.so"; fi
    tag=${lib}_$(echo "$cfg" | tr " =/" "_+-")
    env $cfg timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-extras --no-cpu $EXTRA_ARGS > gpurun_out/ab_${tag}.log 2>&1 || { tail -5 gpurun_out/ab_${tag}.log; exit 1; }
    python -c "import json;d=json.loads(open('gpurun_out/ab_${tag}.log').read().strip().splitlines()[-1]);p=d['roofline']['passes'];print('$lib $cfg', d['value'], d['ms_per_step'], 'ro', p['read_only_pass']['avg_ms'], 'wb', p['write_back_pass']['avg_ms'], p['read_only_pass'].get('avg_ms_by_pending_depth'), 'ext', p['read_only_pass'].get('avg_ms_by_pending_depth_ext'))"
  done
done
