# round-3: new write-back kernel (k_pass_w) + device sweep1site: parity, then timings
set -e
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_sweep_small.py tests/test_gpu_native_sweep.py tests/test_config_golden.py tests/test_gpu_parity.py tests/test_gpu_shadow.py tests/test_gpu_benchsizes.py -q -x --timeout 300 --timeout-method thread -m gpu > gpurun_out/r03d_tests.log 2>&1
timeout -k 10 200 python -u bench.py --no-extras --no-cpu --steps 10 --warmup 2 > gpurun_out/r03d_bench_w.json 2> gpurun_out/r03d_bench_w.err
TCI_PASS_W=0 timeout -k 10 200 python -u bench.py --no-extras --no-cpu --steps 10 --warmup 2 > gpurun_out/r03d_bench_x.json 2> gpurun_out/r03d_bench_x.err
timeout -k 10 200 python -u scripts/small_abi_timing.py > gpurun_out/r03d_abi.log 2>&1
echo done
