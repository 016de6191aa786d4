#!/bin/bash
# K5 solve (scripts/k5_prof.py, r = 1024, R = 32768) under TCI_DGEMM_TILE = 0 / 2 / 3, two rounds
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
for rep in 1 2; do
  for t in 0 2 3; do
    echo -n "tile $t: "; TCI_DGEMM_TILE=$t timeout -k 10 120 python -u scripts/k5_prof.py 1024 32768 3 || exit 1
  done
done
