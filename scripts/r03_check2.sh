# round-3: device sweep parity after the LDS scratch, then the small-config breakdown and the
# kernel's phase profile (TCI_SW_PROF variant)
timeout -k 10 400 python -u -m pytest tests/test_gpu_sweep_small.py tests/test_gpu_native_sweep.py tests/test_config_golden.py -q --maxfail=5 --timeout 200 --timeout-method thread -m gpu > gpurun_out/r03_t8_sweep.log 2>&1 || exit 1
timeout -k 10 200 python -u scripts/small_breakdown.py > gpurun_out/r03_t8_breakdown.log 2>&1 || exit 1
TCI_HIP_LIB=$PWD/tensorcrossinterpolation.jl_amd/lib/variants/swprof.so timeout -k 10 200 python -u scripts/small_breakdown.py > gpurun_out/r03_t8_swprof.log 2>&1
