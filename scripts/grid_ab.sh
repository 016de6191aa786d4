#!/bin/bash
# rrLU pass grid A/B (TCI_PASS_GRIDDIV: the pass grid over 1 / 2 / 4 times fewer CUs) at 4096^2 and
# 8192^2, r = 256, the by-shape epoch settings; median of 5 (scripts/ab_shapes.py), two rounds
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
mkdir -p gpurun_out
for rep in 1 2; do
  for d in ${GRID_DIVS:-1 2 4}; do
    TCI_PASS_GRIDDIV=${DIV:-1} TCI_PASS_GRIDX=${GX:-1} GRID_D=$d timeout -k 10 200 python -u scripts/ab_shapes.py --reps 5 --shape 4096x4096x256 --set 10,1 \
        --shape 8192x8192x256 --set 10,2 | sed "s/^/div $d /" || exit 1
  done
done
