# EXT exact examinations: 4 / 8 / 16 pending updates in flight (TCI_EXB) A/B + bitwise parity of
# the 16-deep build; K5 kernel trace of the dense bench
set -e
mkdir -p gpurun_out
T=r03s3c
LIBS="exb4 exb8 exb16" timeout -k 10 400 bash scripts/ab_lib.sh "AB=1" > gpurun_out/${T}_ab_exb.txt 2>&1
TCI_HIP_LIB=$GRAFT_REPO_ROOT/tensorcrossinterpolation.jl_amd/lib/variants/exb16.so timeout -k 10 500 python -u -m pytest tests/test_gpu_benchsizes.py tests/test_gpu_shadow.py tests/test_gpu_rank1024.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_parity_exb16.txt 2>&1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_k5prof -o run -- python3 scripts/dense_bench.py > gpurun_out/${T}_k5prof.log 2>&1
echo done
