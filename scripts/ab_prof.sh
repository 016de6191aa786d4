# round-3: parity of the rrLU suites, then the two-level epoch (nb 10, epochs 3) against the
# single-level scheme (nb 11) on bench.py 8192^2 r=256, then phase profiles of single passes
# (TCI_PASS_PROF builds: pivot 25 of nb 10 / epochs 3 is an EXT pass with PE 26, PS 6)
set -e
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_shadow.py tests/test_gpu_benchsizes.py -x -q --timeout 400 --timeout-method thread > gpurun_out/r03_t4_tests.log 2>&1
for cfg in "10 3" "11 1" "10 3" "11 1"; do
  set -- $cfg
  timeout -k 10 200 python -u bench.py --no-extras --no-cpu --steps 10 --warmup 2 --nb $1 --epochs $2 >> gpurun_out/r03_t4_nb$1_e$2.json 2>> gpurun_out/r03_t4.err
done
L=$PWD/tensorcrossinterpolation.jl_amd/lib/variants
for K in 24 25; do
  TCI_HIP_LIB=$L/prof$K.so timeout -k 10 200 python -u bench.py --no-extras --no-cpu --steps 1 --warmup 1 --nb 10 --epochs 3 > gpurun_out/r03_t4_prof_K$K.log 2>&1
done
