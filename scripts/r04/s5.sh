# round-4 call 5: A/B of the rrLU pass kernels (HEAD build vs fixed-count memory ops in the MFMA
# search + single-row write-back stores; px4 = timing probe without the single-row stores), the
# parity suites on the new default build, and config 5 as stated against the oracle golden
set -e
mkdir -p gpurun_out
T=r04s5
LIBS="default head px4" bash scripts/ab_lib.sh "TCI_RRLU_EPOCHS=3" > gpurun_out/${T}_ab.txt 2>&1 || { echo "ab rc=$?"; cat gpurun_out/${T}_ab.txt; exit 1; }
cat gpurun_out/${T}_ab.txt
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_shadow.py tests/test_gpu_rank1024.py tests/test_gpu_sharded.py -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_gputest.txt 2>&1 || { echo "gputest rc=$?"; tail -30 gpurun_out/${T}_gputest.txt; exit 1; }
tail -2 gpurun_out/${T}_gputest.txt
timeout -k 10 700 python -u -m pytest tests/test_gpu_c5_as_stated.py -x -v -s --timeout 650 --timeout-method thread > gpurun_out/${T}_c5test.txt 2>&1 || { echo "c5 rc=$?"; tail -30 gpurun_out/${T}_c5test.txt; exit 1; }
tail -5 gpurun_out/${T}_c5test.txt
echo done
