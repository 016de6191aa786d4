set -e
for cfg in "10 3" "10 2" "8 4" "11 1"; do
  set -- $cfg
  timeout -k 10 200 python -u bench.py --no-extras --no-cpu --steps 10 --warmup 2 --nb $1 --epochs $2 > gpurun_out/r03_ab_nb$1_e$2.json 2>> gpurun_out/r03_ab.err
done
