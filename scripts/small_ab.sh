#!/bin/bash
# C3 / C4 A/B of small-sweep settings on one box, alternating: each argument is an env assignment
# list (comma-separated), "-" for the default.   gpurun -- bash scripts/small_ab.sh TAG cfg1 cfg2 ...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
mkdir -p gpurun_out
T=$1; shift
for rep in 1 2; do
  for cfg in "$@"; do
    envs=(); [ "$cfg" != "-" ] && IFS=, read -ra envs <<< "$cfg"
    env "${envs[@]}" TCI2_REPS=5 timeout -k 10 300 python -u scripts/tci2_configs.py C4_qosc40 C3_gauss20d C1_lorentz8d_parity \
        > gpurun_out/${T}_small_${rep}.jsonl 2>&1 || { tail -5 gpurun_out/${T}_small_${rep}.jsonl; exit 1; }
    python - gpurun_out/${T}_small_${rep}.jsonl "$cfg" <<'PY'
import json, sys
for ln in open(sys.argv[1]):
    if ln.startswith("{"):
        d = json.loads(ln)
        print(sys.argv[2], d["config"][:3], "wall_ms", round(d["wall_s"] * 1e3, 2), "lazy_ms", round(d.get("wall_s_lazy", 0) * 1e3, 2))
PY
  done
done
