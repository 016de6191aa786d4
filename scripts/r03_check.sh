# round-3 GPU check: device-resident small sweep, two-level epoch parity, small-config breakdown
timeout -k 10 400 python -u -m pytest tests/test_gpu_sweep_small.py -v --maxfail=5 --timeout 200 --timeout-method thread > gpurun_out/r03_t7_sweep.log 2>&1 || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q --timeout 200 --timeout-method thread -k "two_staging" > gpurun_out/r03_t7_a.log 2>&1 || exit 1
timeout -k 10 500 python -u -m pytest tests/test_gpu_shadow.py -q --timeout 200 --timeout-method thread > gpurun_out/r03_t7_c.log 2>&1 || exit 1
timeout -k 10 200 python -u scripts/small_breakdown.py > gpurun_out/r03_t7_breakdown.log 2>&1
