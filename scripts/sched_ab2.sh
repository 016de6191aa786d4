#!/bin/bash
# Epoch schedule by shape (8-bit shadow build): 4096^2 / 16384^2 (r = 256) and 32768^2 (r = 1024)
#   gpurun -- bash scripts/sched_ab2.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
mkdir -p gpurun_out
T=${1:-sched2}
timeout -k 10 400 python -u scripts/ab_shapes.py --reps 5 --shape 4096x4096x256 --shape 16384x16384x256 \
    --set 10,1 --set 10,2 --set 11,2 --set 12,2 --set 10,3 > gpurun_out/${T}_sched_4k16k.jsonl 2>&1 \
    || { tail -5 gpurun_out/${T}_sched_4k16k.jsonl; exit 1; }
cat gpurun_out/${T}_sched_4k16k.jsonl
timeout -k 10 600 python -u scripts/ab_shapes.py --reps 3 --shape 32768x32768x1024 \
    --set 10,2 --set 11,2 --set 12,2 --set 10,3 > gpurun_out/${T}_sched_32k.jsonl 2>&1 \
    || { tail -5 gpurun_out/${T}_sched_32k.jsonl; exit 1; }
cat gpurun_out/${T}_sched_32k.jsonl
