# round-4 call 6: the MFMA search with its certificate after the prefetches and fixed-count chunk
# loads, against the HEAD build (bench 8192^2 + config-2 shapes); the rrLU parity suites on it;
# phase profiles of single passes (TCI_PASS_PROF builds: pivots 94/95 in the first shadow epoch
# after a write-back, 100/101 at the refresh / EXT boundary); the small-sweep profile of C4 / C3
# (TCI_SW_PROF); K3 tile shapes (TCI_DGEMM_TILE); dense parity tests and bench
set -e
mkdir -p gpurun_out
T=r04s6
V=$PWD/tensorcrossinterpolation.jl_amd/lib/variants
LIBS="default head" bash scripts/ab_lib.sh "TCI_RRLU_EPOCHS=3" > gpurun_out/${T}_ab.txt 2>&1 || { echo "ab rc=$?"; cat gpurun_out/${T}_ab.txt; exit 1; }
cat gpurun_out/${T}_ab.txt
for lib in default head; do
  if [ $lib = default ]; then unset TCI_HIP_LIB; else export TCI_HIP_LIB=$V/$lib.so; fi
  timeout -k 10 200 python -u scripts/ab_shapes.py --reps 5 --set 10,1 --set 10,2 --set 10,3 --shape 2048x2048x256 --shape 4096x4096x256 --shape 8192x8192x256 --shape 16384x16384x256 > gpurun_out/${T}_shapes_$lib.jsonl 2>&1 || { echo "shapes $lib failed"; tail -5 gpurun_out/${T}_shapes_$lib.jsonl; exit 1; }
  echo "$lib"; cat gpurun_out/${T}_shapes_$lib.jsonl | cut -c1-200
done
unset TCI_HIP_LIB
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_shadow.py tests/test_gpu_rank1024.py tests/test_gpu_sharded.py tests/test_gpu_benchsizes.py -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_gputest.txt 2>&1 || { echo "gputest rc=$?"; tail -30 gpurun_out/${T}_gputest.txt; exit 1; }
tail -2 gpurun_out/${T}_gputest.txt
for K in 94 100; do
  lib=pprof$K; [ $K = 100 ] && lib=pprof
  TCI_HIP_LIB=$V/$lib.so timeout -k 10 200 python -u bench.py --no-extras --no-cpu --steps 1 --warmup 1 --epochs 3 > gpurun_out/${T}_pprof$K.log 2>&1 || { echo "pprof $K failed"; tail -5 gpurun_out/${T}_pprof$K.log; exit 1; }
  grep "^\[pass\|^  \[k=" gpurun_out/${T}_pprof$K.log || true
done
TCI_HIP_LIB=$V/swprof.so timeout -k 10 200 python -u scripts/tci2_configs.py C4_qosc40 C3_gauss20d C1_lorentz8d_parity > gpurun_out/${T}_swprof.log 2>&1 || { echo "swprof failed"; tail -5 gpurun_out/${T}_swprof.log; exit 1; }
grep "sweep_small\|wall_s" gpurun_out/${T}_swprof.log | cut -c1-400 || true
for t in 0 1 2 3; do
  TCI_DGEMM_TILE=$t timeout -k 10 200 python -u scripts/dense_bench.py --k3 > gpurun_out/${T}_k3_tile$t.json 2>&1 || { echo "k3 tile $t failed"; tail -5 gpurun_out/${T}_k3_tile$t.json; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/${T}_k3_tile$t.json').read().strip().splitlines()[-1]);print('tile $t', [(r['nb'], r['ms'], r['frac_of_spec']) for r in d['schur_update_k3']])"
done
timeout -k 10 500 python -u -m pytest tests/test_gpu_dense.py -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_densetest.txt 2>&1 || { echo "dense tests rc=$?"; tail -30 gpurun_out/${T}_densetest.txt; exit 1; }
tail -2 gpurun_out/${T}_densetest.txt
timeout -k 10 300 python -u scripts/dense_bench.py > gpurun_out/${T}_dense.json 2>&1 || { echo "dense bench failed"; tail -5 gpurun_out/${T}_dense.json; exit 1; }
python -c "import json;d=json.loads(open('gpurun_out/${T}_dense.json').read().strip().splitlines()[-1]);print(json.dumps(d['sitetensor_solve_k5']));print(json.dumps(d['luci_factors_k4']))"
echo done
