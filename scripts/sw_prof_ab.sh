#!/bin/bash
# Small-sweep phase profile (TCI_SW_PROF variant, lib/variants/swprof.so) of C4 / C3 under env settings
#   gpurun -- bash scripts/sw_prof_ab.sh TAG cfg1 cfg2 ...   ("-" = default; cfg = comma-separated env)
# prints, per setting, the per-bond phase split averaged over the launches of each configuration
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
mkdir -p gpurun_out
T=$1; shift
i=0
for cfg in "$@"; do
  i=$((i + 1))
  envs=(); [ "$cfg" != "-" ] && IFS=, read -ra envs <<< "$cfg"
  env "${envs[@]}" TCI2_REPS=1 TCI_HIP_LIB=$PWD/tensorcrossinterpolation.jl_amd/lib/variants/swprof.so timeout -k 10 200 \
      python -u scripts/tci2_configs.py C4_qosc40 C3_gauss20d > gpurun_out/${T}_swprof$i.log 2>&1 || { tail -20 gpurun_out/${T}_swprof$i.log; exit 1; }
  echo "== $cfg"
  python3 - gpurun_out/${T}_swprof$i.log <<'PY'
import re, sys, collections
acc = collections.defaultdict(list)
for ln in open(sys.argv[1]):
    m = re.match(r"\[sweep_small\] (\d+) bonds (\d+) pivots: (.*) us per bond", ln)
    if m:
        acc[int(m.group(1))].append([float(x) for x in re.findall(r"[\d.]+", m.group(3))])
    m = re.match(r"\[sweep_small\] shader clock [\d.]+ GHz over ([\d.]+) us", ln)
    if m and acc:
        last = max(acc, key=lambda k: len(acc[k]))
import subprocess
print(subprocess.run(["grep", "-c", "prefetched [1-9]", sys.argv[1]], capture_output=True, text=True).stdout.strip(), "launches with prefetched bonds;",
      subprocess.run(["grep", "-c", "prefetched 0 ", sys.argv[1]], capture_output=True, text=True).stdout.strip(), "without")
names = "union staging Pi states loop maxabs rrLU select".split()
for b, rows in sorted(acc.items()):
    avg = [sum(c) / len(c) for c in zip(*rows)]
    print(f"{b} bonds x{len(rows)}:", " ".join(f"{n} {v:.2f}" for n, v in zip(names, avg)))
PY
done
