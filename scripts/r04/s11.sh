# round-4 call 11: phase profile with the late-workgroup report (pivots 95/96), rocprofv3 kernel
# trace + PMC passes of the default bench command on the built commit (scripts/profile_round.sh),
# rrLU parity suites
set -e
mkdir -p gpurun_out
T=r04s11
V=$PWD/tensorcrossinterpolation.jl_amd/lib/variants
TCI_HIP_LIB=$V/pprof95.so timeout -k 10 200 python -u bench.py --no-extras --no-cpu --steps 1 --warmup 1 --epochs 3 > gpurun_out/${T}_pprof95.log 2>&1 || { echo "pprof failed"; tail -5 gpurun_out/${T}_pprof95.log; exit 1; }
grep "^\[pass\|^  \[k=" gpurun_out/${T}_pprof95.log | head -16 || true
timeout -k 10 900 bash scripts/profile_round.sh gpurun_out/${T}_prof > gpurun_out/${T}_prof.log 2>&1 || { echo "profile rc=$?"; tail -20 gpurun_out/${T}_prof.log; exit 1; }
tail -3 gpurun_out/${T}_prof.log
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_shadow.py tests/test_gpu_rank1024.py tests/test_gpu_benchsizes.py tests/test_gpu_sharded.py tests/test_gpu_dense.py -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_gputest.txt 2>&1 || { echo "gputest rc=$?"; tail -30 gpurun_out/${T}_gputest.txt; exit 1; }
tail -2 gpurun_out/${T}_gputest.txt
echo done
