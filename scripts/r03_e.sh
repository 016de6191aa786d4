# round-3: full GPU suite (lazy native set sync, device sweep1site, K3 C prefetch), small-config timeline, full default bench
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03e_gputest.txt 2>&1
timeout -k 10 200 python -u scripts/small_abi_timing.py > gpurun_out/r03e_abi.log 2>&1
timeout -k 10 400 python -u bench.py > gpurun_out/r03e_bench_full.json 2> gpurun_out/r03e_bench_full.err
echo done
