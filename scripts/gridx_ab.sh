#!/bin/bash
# rrLU pass grid A/B: TCI_PASS_GRIDX = 1 / 2 / 3 workgroups per CU at 4096^2 and 8192^2, r = 256
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
for rep in 1 2; do
  for gx in 1 2 3; do
    TCI_PASS_GRIDX=$gx timeout -k 10 200 python -u scripts/ab_shapes.py --reps 5 --shape 4096x4096x256 --set 10,1 \
        --shape 8192x8192x256 --set 10,2 | sed "s/^/gridx $gx /" || exit 1
  done
done
