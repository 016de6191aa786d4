# round-3 A/B: write-back column groups (128 default vs 256: variants/xs256.so) at 8192^2, and the
# epoch depth at 4096^2 (config 2) / 8192^2
set -e
mkdir -p gpurun_out/r03f
B="timeout -k 10 200 python -u bench.py --no-extras --no-cpu --steps 10 --warmup 2"
$B > gpurun_out/r03f/x128.json 2>> gpurun_out/r03f/err.log
TCI_HIP_LIB=$PWD/tensorcrossinterpolation.jl_amd/lib/variants/xs256.so $B > gpurun_out/r03f/x256.json 2>> gpurun_out/r03f/err.log
for cfg in "10 3" "10 2" "10 1" "11 1" "8 1"; do
  set -- $cfg
  $B --m 4096 --n 4096 --nb $1 --epochs $2 > gpurun_out/r03f/c2_nb$1_e$2.json 2>> gpurun_out/r03f/err.log
done
for cfg in "10 2" "11 1"; do
  set -- $cfg
  $B --nb $1 --epochs $2 > gpurun_out/r03f/c8k_nb$1_e$2.json 2>> gpurun_out/r03f/err.log
done
echo done
