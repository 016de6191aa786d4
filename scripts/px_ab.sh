#!/bin/bash
# Kernel-trace A/B of library variants (lib/variants/NAME.so, "default" = lib/libtci_hip.so) on the
# default bench: per variant the average duration of the deep write-back (k_pass_x<1,512>), the
# read-only passes and the bench step, two alternating rounds.
#   gpurun -- bash scripts/px_ab.sh TAG default xu8 ...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
R=$PWD
mkdir -p gpurun_out
T=$1; shift
for rep in 1 2; do
  for lib in "$@"; do
    if [ "$lib" = default ]; then unset TCI_HIP_LIB; else export TCI_HIP_LIB="$R/tensorcrossinterpolation.jl_amd/lib/variants/$lib.so"; fi
    d="$R/gpurun_out/${T}_${lib}_$rep"
    ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$d" -o run \
        -- python3 "$R/bench.py" --steps 5 --warmup 1 --no-extras --no-cpu ) > "$d.log" 2>&1 || { tail -20 "$d.log"; exit 1; }
    python3 - "$d" "$lib" <<'PY'
import csv, glob, json, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
wb = ro = ron = 0.0
for r in csv.DictReader(open(f)):
    n = r["Name"]
    if n.startswith("void tci::k_pass_x<1, 512>"):
        wb = float(r["AverageNs"]) / 1e3
    if n.startswith("void tci::k_pass_mf<") and ", false>" in n and "true, false>" not in n.replace("false, true, false", ""):
        pass
    if n.startswith("void tci::k_pass_mf<") and n.split("<")[1].split(",")[2].strip() == "false":
        ro += float(r["TotalDurationNs"]) / 1e3
        ron += int(r["Calls"])
step = None
for ln in open(sys.argv[1] + ".log"):
    if ln.startswith("{"):
        step = json.loads(ln)["ms_per_step"]
print(f"{sys.argv[2]:12s} write-back {wb:7.1f} us  read-only avg {ro / max(ron, 1):6.2f} us  step {step} ms")
PY
  done
done
