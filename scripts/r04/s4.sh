# round-4 call 4: deep write-back with fixed-count buffer memory ops (precise vmcnt waits):
# parity suites that run it, the default bench line, and the C5 oracle's last half-sweep + final
# sweep1site in the background
set -e
mkdir -p gpurun_out
T=r04s4
rm -rf gpurun_out/c5state && cp -r oracle/_ckpt/c5 gpurun_out/c5state
OMP_NUM_THREADS=14 timeout -k 10 1100 python -u tests/golden/make_c5_golden.py --state gpurun_out/c5state --halves 1 > gpurun_out/${T}_c5.log 2>&1 &
OPID=$!
timeout -k 10 300 python -u bench.py --no-extras --no-cpu --steps 10 --warmup 2 > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_shadow.py tests/test_gpu_rank1024.py tests/test_gpu_sharded.py tests/test_gpu_benchsizes.py -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_gputest.txt 2>&1 || echo "gputest rc=$?" >> gpurun_out/${T}_gputest.txt
while kill -0 $OPID 2>/dev/null; do sleep 30; date >> gpurun_out/${T}_hb.txt; done
wait $OPID; echo "oracle rc=$?" >> gpurun_out/${T}_c5.log
tail -3 gpurun_out/${T}_gputest.txt
cp tests/golden/c5_golden.json gpurun_out/c5_golden.json 2>/dev/null || true
echo done
