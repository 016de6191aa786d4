#!/bin/bash
# Kernel trace (rocprofv3 --kernel-trace --stats) of the C4 / C3 TCI2 runs under env settings:
#   gpurun -- bash scripts/sw_trace_ab.sh TAG cfg1 cfg2 ...   ("-" = default; cfg = comma-separated env)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
R=$PWD
mkdir -p gpurun_out
T=$1; shift
i=0
for cfg in "$@"; do
  i=$((i + 1))
  envs=(); [ "$cfg" != "-" ] && IFS=, read -ra envs <<< "$cfg"
  for e in "${envs[@]}"; do export "$e"; done
  ( cd /tmp && export TMPDIR=/tmp TCI2_REPS=3 && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
      -d "$R/gpurun_out/${T}_trace$i" -o run -- python3 "$R/scripts/tci2_configs.py" C4_qosc40 C3_gauss20d ) \
      > gpurun_out/${T}_trace$i.log 2>&1 || { tail -20 gpurun_out/${T}_trace$i.log; exit 1; }
  for e in "${envs[@]}"; do unset "${e%%=*}"; done
  echo "== $cfg"
  grep '^{' gpurun_out/${T}_trace$i.log | cut -c1-120
  f=$(find gpurun_out/${T}_trace$i -name '*kernel_stats.csv' | sed -n 1p) || true
  [ -n "$f" ] && cut -d, -f1-6 "$f" | cut -c1-160 | sed -n 1,14p
done
exit 0
