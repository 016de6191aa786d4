#!/bin/bash
# Profiles of the default bench command for profiles/ (run on the GPU box from the repo root):
#   1. rocprofv3 --kernel-trace --stats           -> OUT/trace
#   2. one rocprofv3 --pmc pass per counter group -> OUT/pmc1.. (FETCH_SIZE and WRITE_SIZE apart,
#      as MI355X_MICROARCH.md prescribes), summarised into OUT/pmc_summary.json
# Usage: scripts/profile_round.sh OUT [bench args...]   (default bench args: --steps 3 --warmup 1)
set -e
OUT=$1; shift
ARGS=${*:-"--steps 3 --warmup 1 --no-extras --no-cpu"}
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$OUT/trace" -o run -- \
  python3 "$R/bench.py" $ARGS > "$R/$OUT/trace.log" 2>&1 || { echo "kernel trace failed"; tail -5 "$R/$OUT/trace.log"; exit 1; }
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" ${EXTRA_PMC_GROUPS}; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d "$R/$OUT/pmc$i" -o run -- \
    python3 "$R/bench.py" $ARGS > "$R/$OUT/pmc$i.log" 2>&1 || { echo "pmc group $i failed"; tail -5 "$R/$OUT/pmc$i.log"; exit 1; }
done
python3 "$R/scripts/pmc_summary.py" "$R/$OUT" "$R/$OUT/pmc_summary.json"
echo done
