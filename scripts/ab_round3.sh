# round-3 A/B: two-level epoch and the XCD-class ticket (bench.py, 8192^2 r=256), after the parity tests
set -e
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_shadow.py tests/test_gpu_benchsizes.py tests/test_gpu_sharded.py -x -q --timeout 400 --timeout-method thread > gpurun_out/r03_t3_tests.log 2>&1
for cfg in "10 3" "11 1"; do
  set -- $cfg
  timeout -k 10 200 python -u bench.py --no-extras --no-cpu --steps 10 --warmup 2 --nb $1 --epochs $2 > gpurun_out/r03_t3_nb$1_e$2.json 2>> gpurun_out/r03_t3.err
done
TCI_HIP_LIB=$PWD/tensorcrossinterpolation.jl_amd/lib/variants/ticket1.so timeout -k 10 200 python -u bench.py --no-extras --no-cpu --steps 10 --warmup 2 --nb 11 --epochs 1 > gpurun_out/r03_t3_ticket1_nb11_e1.json 2>> gpurun_out/r03_t3.err
