#!/bin/bash
# K3 tile-shape A/B (scripts/k3_tiles.py) over TCI_DGEMM_TILE = 0 / 1 / 2 / 3, two rounds
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
mkdir -p gpurun_out
for rep in 1 2; do
  for t in 0 1 2 3; do
    TCI_DGEMM_TILE=$t timeout -k 10 120 python -u scripts/k3_tiles.py || exit 1
  done
done
