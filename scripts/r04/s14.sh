# round-4 call 14: the grid-wide examination bound as a variant (gridtau.so): A/B against the
# default build, the rrLU parity suites and config 5 on the variant; then the full -m gpu suite,
# and smoke() of the default build
set -e
mkdir -p gpurun_out
T=r04s14
V=$PWD/tensorcrossinterpolation.jl_amd/lib/variants
LIBS="default gridtau" bash scripts/ab_lib.sh "TCI_RRLU_EPOCHS=3" > gpurun_out/${T}_ab.txt 2>&1 || { echo "ab rc=$?"; cat gpurun_out/${T}_ab.txt; exit 1; }
cat gpurun_out/${T}_ab.txt
TCI_HIP_LIB=$V/gridtau.so timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_shadow.py tests/test_gpu_rank1024.py tests/test_gpu_benchsizes.py tests/test_gpu_sharded.py tests/test_gpu_c5_as_stated.py -x -q --timeout 650 --timeout-method thread > gpurun_out/${T}_gputest_gridtau.txt 2>&1 || { echo "gridtau gputest rc=$?"; tail -30 gpurun_out/${T}_gputest_gridtau.txt; exit 1; }
tail -2 gpurun_out/${T}_gputest_gridtau.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_gputest.txt 2>&1 || { echo "gputest rc=$?"; tail -30 gpurun_out/${T}_gputest.txt; exit 1; }
tail -2 gpurun_out/${T}_gputest.txt
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${T}_smoke.txt 2>&1 || { echo "smoke rc=$?"; tail -20 gpurun_out/${T}_smoke.txt; exit 1; }
tail -1 gpurun_out/${T}_smoke.txt
echo done
