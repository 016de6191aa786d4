# round-4 call 17: the deep write-back drains before requesting the next chunk (pxdrain.so): A/B against the
# default build; the rrLU parity suites and config 5 on the variant only if its step is faster
set -e
mkdir -p gpurun_out
T=r04s17
V=$PWD/tensorcrossinterpolation.jl_amd/lib/variants
LIBS="default pxdrain" bash scripts/ab_lib.sh "TCI_RRLU_EPOCHS=3" > gpurun_out/${T}_ab.txt 2>&1 || { echo "ab rc=$?"; cat gpurun_out/${T}_ab.txt; exit 1; }
cat gpurun_out/${T}_ab.txt
if awk '$1=="default"{d=$4} $1=="pxdrain"{v=$4} END{exit !(v<d)}' gpurun_out/${T}_ab.txt; then :; else echo "pxdrain not faster: no parity run"; exit 0; fi
TCI_HIP_LIB=$V/pxdrain.so timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_shadow.py tests/test_gpu_rank1024.py tests/test_gpu_benchsizes.py tests/test_gpu_sharded.py tests/test_gpu_c5_as_stated.py -x -q --timeout 650 --timeout-method thread > gpurun_out/${T}_gputest_pxdrain.txt 2>&1 || { echo "pxdrain gputest rc=$?"; tail -30 gpurun_out/${T}_gputest_pxdrain.txt; exit 1; }
tail -2 gpurun_out/${T}_gputest_pxdrain.txt
echo done
