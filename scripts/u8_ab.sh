#!/bin/bash
# The 8-bit shadow variant (lib/variants/u8.so: make variant NAME=u8 VFLAGS=-DTCI_SH_U8=1) against
# the default build on the GPU box: the rrLU parity suites on the variant, the bench A/B, the shapes
# A/B (4096^2 / 16384^2 at the by-shape epoch schedule), and config 5 as stated on the variant.
#   gpurun --timeout 1200 -- bash scripts/u8_ab.sh TAG [c5]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
mkdir -p gpurun_out
T=${1:-u8}
U8=$PWD/tensorcrossinterpolation.jl_amd/lib/variants/u8.so
echo "[$T] parity suites on u8 ($(date +%T))"
TCI_HIP_LIB=$U8 timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    -k "shadow or benchsizes or parity or rank1024 or rrlu_copy or sharded_one_rank" > gpurun_out/${T}_u8_gputest.txt 2>&1 \
    || { tail -30 gpurun_out/${T}_u8_gputest.txt; exit 1; }
tail -2 gpurun_out/${T}_u8_gputest.txt
echo "[$T] bench A/B ($(date +%T))"
LIBS="default u8 default u8" timeout -k 10 600 bash scripts/ab_lib.sh A=1 > gpurun_out/${T}_ab.txt 2>&1 || { cat gpurun_out/${T}_ab.txt; exit 1; }
cat gpurun_out/${T}_ab.txt
echo "[$T] shapes ($(date +%T))"
for lib in default u8; do
  if [ $lib = u8 ]; then export TCI_HIP_LIB=$U8; else unset TCI_HIP_LIB; fi
  timeout -k 10 300 python -u scripts/ab_shapes.py --reps 5 --set 10,0 --shape 4096x4096x256 --shape 16384x16384x256 \
      > gpurun_out/${T}_shapes_$lib.jsonl 2>&1 || { tail -5 gpurun_out/${T}_shapes_$lib.jsonl; exit 1; }
  sed "s/^/$lib /" gpurun_out/${T}_shapes_$lib.jsonl
done
unset TCI_HIP_LIB
if [ "$2" = c5 ]; then
  echo "[$T] config 5 as stated on u8 ($(date +%T))"
  TCI_HIP_LIB=$U8 TCI2_C5_LAZY=0 timeout -k 10 400 python -u scripts/tci2_configs.py C5_cp12d_K1024 > gpurun_out/${T}_u8_c5.jsonl 2>&1 \
      || { tail -5 gpurun_out/${T}_u8_c5.jsonl; exit 1; }
  tail -c 600 gpurun_out/${T}_u8_c5.jsonl
fi
echo "[$T] done ($(date +%T))"
