# round-4 call 3: deep write-back LDS probes (timing-only variants, wrong values) and the sharded
# rrLU tests (two-level epoch in the sharded driver) while the C5 oracle runs half-sweep 5 on the
# host CPU in the background
set -e
mkdir -p gpurun_out
T=r04s3
rm -rf gpurun_out/c5state && cp -r oracle/_ckpt/c5 gpurun_out/c5state
OMP_NUM_THREADS=15 timeout -k 10 1000 python -u tests/golden/make_c5_golden.py --state gpurun_out/c5state --halves 1 > gpurun_out/${T}_c5.log 2>&1 &
OPID=$!
LIBS="default pxexp1 pxexp2 pxexp3" bash scripts/ab_lib.sh "TCI_RRLU_EPOCHS=3" > gpurun_out/${T}_ab_px.txt 2>&1 || echo "ab rc=$?" >> gpurun_out/${T}_ab_px.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_sharded.py tests/test_distributed.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${T}_gputest.txt 2>&1 || echo "gputest rc=$?" >> gpurun_out/${T}_gputest.txt
while kill -0 $OPID 2>/dev/null; do sleep 30; date >> gpurun_out/${T}_hb.txt; done
wait $OPID; echo "oracle rc=$?" >> gpurun_out/${T}_c5.log
cat gpurun_out/${T}_ab_px.txt
tail -3 gpurun_out/${T}_gputest.txt
echo done
