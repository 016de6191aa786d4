# K5 register-panel getrf: parity + timing; read-only pass timing split by EXT / first shadow epoch
set -e
mkdir -p gpurun_out
T=r03s3b
timeout -k 10 300 python -u -m pytest tests/test_gpu_dense.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_dense_tests.txt 2>&1
timeout -k 10 200 python -u bench.py --no-extras --no-cpu --steps 10 --warmup 2 > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err
timeout -k 10 300 python -u scripts/dense_bench.py > gpurun_out/${T}_dense.json 2>&1
echo done
