#!/bin/bash
# Exact examinations and certificate failures per rrLU pass: the bench
# factorisation (8192^2, r = 256) and the 32768^2 r = 1024 shape on census builds
# (make variant NAME=census VFLAGS="-DTCI_PASS_PROF=27 -DTCI_EXAM_CENSUS" [-DTCI_SH_U8=0 -> census16]).
#   gpurun -- bash scripts/exam_census.sh TAG [lib ...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
mkdir -p gpurun_out
T=${1:-census}; shift
for lib in ${@:-census census16}; do
  TCI_HIP_LIB=$PWD/tensorcrossinterpolation.jl_amd/lib/variants/$lib.so timeout -k 10 300 python -u bench.py --no-extras \
      --no-cpu --steps 1 --warmup 0 > gpurun_out/${T}_$lib.log 2>&1 || { tail -20 gpurun_out/${T}_$lib.log; exit 1; }
  TCI_HIP_LIB=$PWD/tensorcrossinterpolation.jl_amd/lib/variants/$lib.so timeout -k 10 300 python -u scripts/ab_shapes.py \
      --reps 1 --set 10,0 --shape 32768x32768x1024 > gpurun_out/${T}_${lib}_32k.log 2>&1 || { tail -20 gpurun_out/${T}_${lib}_32k.log; exit 1; }
  python scripts/census_summary.py gpurun_out/${T}_$lib.log gpurun_out/${T}_${lib}_32k.log > gpurun_out/${T}_${lib}_summary.json
  cat gpurun_out/${T}_${lib}_summary.json
done
