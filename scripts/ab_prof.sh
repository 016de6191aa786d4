# round-3 phase profiles of single passes (TCI_PASS_PROF builds): EXT pass of the two-level
# epoch (nb 10, epochs 3: pivot 25 has PE 26 / PS 6) against the single-level pass (nb 11)
set -e
L=$PWD/tensorcrossinterpolation.jl_amd/lib/variants
for cfg in "10 3" "11 1"; do
  set -- $cfg
  for K in 24 25; do
    TCI_HIP_LIB=$L/prof$K.so timeout -k 10 200 python -u bench.py --no-extras --no-cpu --steps 1 --warmup 1 --nb $1 --epochs $2 > gpurun_out/r03_prof_nb$1_e$2_K$K.log 2>&1
  done
done
