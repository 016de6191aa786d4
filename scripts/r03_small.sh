# round-3: small-config parity after a sweep-kernel change, then the host ABI timeline and the
# same under a kernel trace
set -e
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_sweep_small.py tests/test_gpu_native_sweep.py tests/test_config_golden.py -q -x --timeout 200 --timeout-method thread -m gpu > gpurun_out/r03c_tests.log 2>&1
timeout -k 10 200 python -u scripts/small_abi_timing.py > gpurun_out/r03c_abi.log 2>&1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03c_trace -o run -- python3 scripts/small_abi_timing.py > gpurun_out/r03c_trace.log 2>&1
echo done
