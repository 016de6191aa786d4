# K5 getrf panel A/B (TCI_GETRF_NT = 1024 / 256 threads per register panel): the dense parity tests
# on the 256-thread form, then the dense bench (K5 solve timings) for both.   gpurun -- bash scripts/k5_ab.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
T=${1:-k5}
TCI_GETRF_NT=256 timeout -k 10 600 python -u -m pytest tests/test_gpu_dense.py -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/${T}_densetest.txt 2>&1 || { tail -30 gpurun_out/${T}_densetest.txt; exit 1; }
tail -2 gpurun_out/${T}_densetest.txt
for nt in 1024 256 1024 256; do
  TCI_GETRF_NT=$nt timeout -k 10 300 python -u scripts/dense_bench.py > gpurun_out/${T}_dense_$nt.json 2>&1 || { tail -5 gpurun_out/${T}_dense_$nt.json; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/${T}_dense_$nt.json').read().strip().splitlines()[-1]);print('NT $nt', json.dumps([(x['r'], x['R'], x['mfma']['ms']) for x in d['sitetensor_solve_k5']]))"
done
