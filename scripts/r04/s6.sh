# round-4 call 6: phase profiles of single rrLU passes (TCI_PASS_PROF builds: pivots 94/95 of the
# first shadow epoch after a write-back, 100/101 at the refresh / EXT boundary), the small-sweep
# profile of C4 / C3 (TCI_SW_PROF build), K3 tile-shape A/B (TCI_DGEMM_TILE), the dense parity
# tests (preloaded-interchange getrf swap) and the dense bench
set -e
mkdir -p gpurun_out
T=r04s6
V=$PWD/tensorcrossinterpolation.jl_amd/lib/variants
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
timeout -k 10 600 python -u -m pytest tests/test_gpu_dense.py -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_densetest.txt 2>&1 || { echo "dense tests rc=$?"; tail -30 gpurun_out/${T}_densetest.txt; exit 1; }
tail -2 gpurun_out/${T}_densetest.txt
timeout -k 10 400 python -u scripts/dense_bench.py > gpurun_out/${T}_dense.json 2>&1 || { echo "dense bench failed"; tail -5 gpurun_out/${T}_dense.json; exit 1; }
python -c "import json;d=json.loads(open('gpurun_out/${T}_dense.json').read().strip().splitlines()[-1]);print(json.dumps(d['sitetensor_solve_k5']));print(json.dumps(d['luci_factors_k4']))"
echo done
