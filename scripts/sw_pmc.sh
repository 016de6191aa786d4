#!/bin/bash
# PMC passes (one rocprofv3 --pmc run per argument, counters space-separated) over the C4 TCI2 run,
# summed over the k_sweep_small launches:   gpurun -- bash scripts/sw_pmc.sh TAG "C1 C2" "C3 C4" ...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
R=$PWD
mkdir -p gpurun_out
T=$1; shift
i=0
for ctrs in "$@"; do
  i=$((i + 1))
  ( cd /tmp && export TMPDIR=/tmp TCI2_REPS=1 && timeout -s KILL 120 rocprofv3 --pmc $ctrs --output-format csv \
      -d "$R/gpurun_out/${T}_pmc$i" -o run -- python3 "$R/scripts/tci2_configs.py" C4_qosc40 ) \
      > gpurun_out/${T}_pmc$i.log 2>&1 || { tail -20 gpurun_out/${T}_pmc$i.log; exit 1; }
  f=$(find gpurun_out/${T}_pmc$i -name '*counter_collection.csv' | sed -n 1p) || true
  [ -n "$f" ] && python3 - "$f" "$ctrs" <<'PY'
import csv, sys, collections
acc = collections.defaultdict(float)
n = collections.Counter()
for r in csv.DictReader(open(sys.argv[1])):
    k = r["Kernel_Name"]
    if "k_sweep_small" not in k:
        continue
    acc[r["Counter_Name"]] += float(r["Counter_Value"])
    n[r["Counter_Name"]] += 1
print(sys.argv[2], {c: (round(v), n[c]) for c, v in acc.items()})
PY
done
exit 0
