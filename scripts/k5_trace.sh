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
f=$(find gpurun_out/${T}_k5 -name '*kernel_trace.csv' | sed -n 1p)
python3 - "$f" <<'PY'
import csv, sys
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
# the last solve: from its k_transpose_sq to the end
idx = [i for i, r in enumerate(rows) if "k_transpose_sq" in r["Kernel_Name"]]
seg = rows[idx[-1]:]
t0, t1 = int(seg[0]["Start_Timestamp"]), int(seg[-1]["End_Timestamp"])
busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in seg)
print(f"last solve: {len(seg)} kernels, span {(t1 - t0) / 1e3:.1f} us, busy {busy / 1e3:.1f} us, idle {(t1 - t0 - busy) / 1e3:.1f} us")
gaps = [(int(b["Start_Timestamp"]) - int(a["End_Timestamp"])) / 1e3 for a, b in zip(seg, seg[1:])]
print("gap quantiles (us):", [round(sorted(gaps)[int(q * (len(gaps) - 1))], 2) for q in (0.1, 0.5, 0.9, 0.99)])
PY
