# round-3: host ABI timeline of the small configs, then the same under a kernel trace
set -e
mkdir -p gpurun_out
timeout -k 10 200 python -u scripts/small_abi_timing.py > gpurun_out/r03c_abi.log 2>&1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03c_trace -o run -- python3 scripts/small_abi_timing.py > gpurun_out/r03c_trace.log 2>&1
echo done
