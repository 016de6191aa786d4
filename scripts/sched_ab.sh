#!/bin/bash
# Epoch schedule A/B of the 8-bit shadow build (nb pivots per shadow epoch, epochs shadow epochs per
# exact epoch, nb * epochs <= 31): 8192^2 r = 256 and 32768^2 r = 1024, median of reps.
#   gpurun -- bash scripts/sched_ab.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
mkdir -p gpurun_out
T=${1:-sched}
timeout -k 10 400 python -u scripts/ab_shapes.py --reps 5 --shape 8192x8192x256 \
    --set 10,3 --set 8,3 --set 9,3 --set 7,4 --set 6,5 --set 11,2 --set 15,2 --set 10,2 > gpurun_out/${T}_sched_8k.jsonl 2>&1 \
    || { tail -5 gpurun_out/${T}_sched_8k.jsonl; exit 1; }
cat gpurun_out/${T}_sched_8k.jsonl
timeout -k 10 600 python -u scripts/ab_shapes.py --reps 3 --shape 32768x32768x1024 \
    --set 10,3 --set 8,3 --set 7,4 --set 6,5 --set 15,2 > gpurun_out/${T}_sched_32k.jsonl 2>&1 \
    || { tail -5 gpurun_out/${T}_sched_32k.jsonl; exit 1; }
cat gpurun_out/${T}_sched_32k.jsonl
