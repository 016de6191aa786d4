# round-4 call 2: full bench line (extras: rrlu_configs with the by-shape epoch schedule), then the
# C5 oracle half-sweep 4 on the host CPU in the background while the new GPU tests run
set -e
mkdir -p gpurun_out
T=r04s2
timeout -k 10 500 python -u bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err
rm -rf gpurun_out/c5state && cp -r oracle/_ckpt/c5 gpurun_out/c5state
OMP_NUM_THREADS=15 timeout -k 10 1000 python -u tests/golden/make_c5_golden.py --state gpurun_out/c5state --halves 1 > gpurun_out/${T}_c5.log 2>&1 &
OPID=$!
timeout -k 10 600 python -u -m pytest tests/test_gpu_contraction.py tests/test_gpu_complex.py tests/test_gpu_hostfunction.py -x -v --timeout 300 --timeout-method thread > gpurun_out/${T}_gputest.txt 2>&1 || echo "gputest rc=$?" >> gpurun_out/${T}_gputest.txt
while kill -0 $OPID 2>/dev/null; do sleep 30; date >> gpurun_out/${T}_hb.txt; done
wait $OPID; echo "oracle rc=$?" >> gpurun_out/${T}_c5.log
tail -3 gpurun_out/${T}_gputest.txt
echo done
