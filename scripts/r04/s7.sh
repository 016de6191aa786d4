# round-4 call 7: phase profiles with thread 0's sub-phases (pivots 95/96: first shadow epoch,
# 105/106: EXT), the A/B of the current MFMA search (dead last-trip approx skipped in first-epoch
# passes) against the HEAD build over shapes, and the rrLU parity suites
set -e
mkdir -p gpurun_out
T=r04s7
V=$PWD/tensorcrossinterpolation.jl_amd/lib/variants
for K in 95 105; do
  TCI_HIP_LIB=$V/pprof$K.so timeout -k 10 200 python -u bench.py --no-extras --no-cpu --steps 1 --warmup 1 --epochs 3 > gpurun_out/${T}_pprof$K.log 2>&1 || { echo "pprof $K failed"; tail -5 gpurun_out/${T}_pprof$K.log; exit 1; }
  grep "^\[pass\|^  \[k=" gpurun_out/${T}_pprof$K.log || true
done
for lib in default head; do
  if [ $lib = default ]; then unset TCI_HIP_LIB; else export TCI_HIP_LIB=$V/$lib.so; fi
  timeout -k 10 200 python -u scripts/ab_shapes.py --reps 7 --set 10,1 --set 10,3 --shape 2048x2048x256 --shape 4096x4096x256 --shape 8192x8192x256 > gpurun_out/${T}_shapes_$lib.jsonl 2>&1 || { echo "shapes $lib failed"; tail -5 gpurun_out/${T}_shapes_$lib.jsonl; exit 1; }
  echo "$lib"; cat gpurun_out/${T}_shapes_$lib.jsonl
done
unset TCI_HIP_LIB
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_shadow.py tests/test_gpu_rank1024.py tests/test_gpu_benchsizes.py -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_gputest.txt 2>&1 || { echo "gputest rc=$?"; tail -30 gpurun_out/${T}_gputest.txt; exit 1; }
tail -2 gpurun_out/${T}_gputest.txt
echo done
