#!/bin/bash
# kernel trace of the K5 solve at the C5 shape (scripts/k5_prof.py)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
R=$PWD
mkdir -p gpurun_out
T=$1
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/${T}_k5" -o run \
    -- python3 "$R/scripts/k5_prof.py" 1024 32768 3 ) > gpurun_out/${T}_k5.log 2>&1 || { tail -20 gpurun_out/${T}_k5.log; exit 1; }
grep "per solve" gpurun_out/${T}_k5.log
f=$(find gpurun_out/${T}_k5 -name '*kernel_stats.csv' | sed -n 1p)
python3 - "$f" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    print(f'{r["Name"][:70]:72s} {int(r["Calls"]):6d} {float(r["TotalDurationNs"]) / 4e6:9.3f} ms/solve {float(r["AverageNs"]) / 1e3:9.2f} us avg')
PY
