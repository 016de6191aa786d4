# round-3 session-3: K5 parity first (register panel, readlane pivot row, preloaded interchanges),
# then the final evidence (scripts/r03_s3_final.sh)
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_dense.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03s3e_dense_tests.txt 2>&1
bash scripts/r03_s3_final.sh
