#!/bin/bash
# C3 / C4 wall time of two library builds on ONE box, alternating: the default
# build against a variant (lib/variants/NAME.so, e.g. j1 = the sources of 8137df7).
#   gpurun -- bash scripts/c4_bisect.sh TAG NAME [rounds]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
mkdir -p gpurun_out
T=${1:-c4}; V=${2:-j1}; N=${3:-2}
for i in $(seq 1 $N); do
  for lib in default $V; do
    if [ $lib = default ]; then unset TCI_HIP_LIB; else export TCI_HIP_LIB=$PWD/tensorcrossinterpolation.jl_amd/lib/variants/$lib.so; fi
    TCI2_REPS=5 timeout -k 10 300 python -u scripts/tci2_configs.py C4_qosc40 C3_gauss20d > gpurun_out/${T}_${lib}_$i.jsonl 2>&1 \
        || { tail -5 gpurun_out/${T}_${lib}_$i.jsonl; exit 1; }
    python - gpurun_out/${T}_${lib}_$i.jsonl $lib <<'PY'
import json, sys
for ln in open(sys.argv[1]):
    if ln.startswith("{"):
        d = json.loads(ln)
        print(sys.argv[2], d["config"][:3], "wall_ms", round(d["wall_s"] * 1e3, 2), "lazy_ms", round(d.get("wall_s_lazy", 0) * 1e3, 2), d["ranks"][-1])
PY
  done
done
