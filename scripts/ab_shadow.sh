#!/bin/bash
# A/B of the rrLU pass variants on the GPU box: deferred depth nb x library variant.
# Prints one line per run: lib nb GFLOP/s ro_ms wb_ms by-pending.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
for lib in ${LIBS:-default}; do
  for nb in ${NBS:-10}; do
    if [ "$lib" = default ]; then unset TCI_HIP_LIB; else export TCI_HIP_LIB="$R/tensorcrossinterpolation.jl_amd/lib/variants/$lib.so"; fi
    TCI_RRLU_NB=$nb timeout -k 10 120 python bench.py --no-extras --no-cpu $EXTRA_ARGS > gpurun_out/ab_${lib}_${nb}.log 2>&1 || { echo "run $lib $nb failed"; tail -3 gpurun_out/ab_${lib}_${nb}.log; exit 1; }
    tail -1 gpurun_out/ab_${lib}_${nb}.log | python3 -c "
import json,sys; d=json.load(sys.stdin); p=d['roofline']['passes']
print('$lib', 'nb=$nb', d['value'], 'ro', p['read_only_pass']['avg_ms'], 'wb', p['write_back_pass']['avg_ms'], p['read_only_pass'].get('avg_ms_by_pending_depth'))"
  done
done
