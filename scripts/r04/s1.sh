# round-4 call 1 on one MI355X: default bench line; then, with the C5 oracle half-sweep running on
# the host CPU in the background (tests/golden/make_c5_golden.py), the epoch-schedule A/B over
# shapes and the GPU suite
set -e
mkdir -p gpurun_out
T=r04s1
timeout -k 10 400 python -u bench.py --no-extras > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err
rm -rf gpurun_out/c5state && cp -r oracle/_ckpt/c5 gpurun_out/c5state
nproc > gpurun_out/${T}_host.txt; (lscpu | head -20) >> gpurun_out/${T}_host.txt || true
OMP_NUM_THREADS=13 timeout -k 10 1000 python -u tests/golden/make_c5_golden.py --state gpurun_out/c5state --halves 1 > gpurun_out/${T}_c5.log 2>&1 &
OPID=$!
timeout -k 10 300 python -u scripts/ab_shapes.py --reps 5 > gpurun_out/${T}_ab_shapes.jsonl 2>&1
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${T}_gputest.txt 2>&1 || echo "gputest rc=$?" >> gpurun_out/${T}_gputest.txt
while kill -0 $OPID 2>/dev/null; do sleep 30; date >> gpurun_out/${T}_hb.txt; done
wait $OPID; echo "oracle rc=$?" >> gpurun_out/${T}_c5.log
tail -3 gpurun_out/${T}_gputest.txt
echo done
