# round-4 call 12: the MFMA search's exact examinations pruned by a grid-wide bound (each
# workgroup publishes its certified seed bound; read once after the seed): A/B vs HEAD build,
# phase profile with the examination counts, rrLU / dense / sharded parity suites, config 5
set -e
mkdir -p gpurun_out
T=r04s12
V=$PWD/tensorcrossinterpolation.jl_amd/lib/variants
LIBS="default head" bash scripts/ab_lib.sh "TCI_RRLU_EPOCHS=3" > gpurun_out/${T}_ab.txt 2>&1 || { echo "ab rc=$?"; cat gpurun_out/${T}_ab.txt; exit 1; }
cat gpurun_out/${T}_ab.txt
for lib in default head; do
  if [ $lib = default ]; then unset TCI_HIP_LIB; else export TCI_HIP_LIB=$V/$lib.so; fi
  timeout -k 10 200 python -u scripts/ab_shapes.py --reps 7 --set 10,1 --set 10,3 --shape 2048x2048x256 --shape 4096x4096x256 --shape 8192x8192x256 > gpurun_out/${T}_shapes_$lib.jsonl 2>&1 || { echo "shapes $lib failed"; tail -5 gpurun_out/${T}_shapes_$lib.jsonl; exit 1; }
  echo "$lib"; python -c "
import json
for l in open('gpurun_out/${T}_shapes_$lib.jsonl'):
    try: d=json.loads(l)
    except Exception: continue
    print(d['m'], d['epochs'], d['ms_median'])"
done
unset TCI_HIP_LIB
TCI_HIP_LIB=$V/pprof95.so timeout -k 10 200 python -u bench.py --no-extras --no-cpu --steps 1 --warmup 1 --epochs 3 > gpurun_out/${T}_pprof95.log 2>&1 || { echo "pprof failed"; tail -5 gpurun_out/${T}_pprof95.log; exit 1; }
grep "^\[pass\|^  \[k=" gpurun_out/${T}_pprof95.log | head -16 || true
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_shadow.py tests/test_gpu_rank1024.py tests/test_gpu_benchsizes.py tests/test_gpu_sharded.py tests/test_gpu_dense.py -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_gputest.txt 2>&1 || { echo "gputest rc=$?"; tail -30 gpurun_out/${T}_gputest.txt; exit 1; }
tail -2 gpurun_out/${T}_gputest.txt
timeout -k 10 700 python -u -m pytest tests/test_gpu_c5_as_stated.py -x -v -s --timeout 650 --timeout-method thread > gpurun_out/${T}_c5test.txt 2>&1 || { echo "c5 rc=$?"; tail -30 gpurun_out/${T}_c5test.txt; exit 1; }
grep "C5 as stated\|passed\|failed" gpurun_out/${T}_c5test.txt
echo done
