# round-3 profiles: small-config breakdown (default and phase-profile builds), then the bench's
# kernel trace + FETCH_SIZE / WRITE_SIZE passes (scripts/profile_round.sh)
set -e
mkdir -p gpurun_out
timeout -k 10 200 python -u scripts/small_breakdown.py > gpurun_out/r03b_breakdown.log 2>&1
TCI_HIP_LIB=$PWD/tensorcrossinterpolation.jl_amd/lib/variants/swprof.so timeout -k 10 200 python -u scripts/small_breakdown.py > gpurun_out/r03b_swprof.log 2>&1
bash scripts/profile_round.sh gpurun_out/prof_r03b
