# K5: register panel with the pivot row broadcast by readlane + preloaded interchanges: parity,
# timing, kernel trace of the dense bench
set -e
mkdir -p gpurun_out
T=r03s3d
timeout -k 10 300 python -u -m pytest tests/test_gpu_dense.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_dense_tests.txt 2>&1
timeout -k 10 300 python -u scripts/dense_bench.py > gpurun_out/${T}_dense.json 2>&1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_k5prof -o run -- python3 scripts/dense_bench.py > gpurun_out/${T}_k5prof.log 2>&1
echo done
