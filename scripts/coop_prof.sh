set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
TCI_HIP_LIB=$PWD/tensorcrossinterpolation.jl_amd/lib/variants/coopprof.so timeout -k 10 120 python -u scripts/k5_prof.py 1024 64 2 > gpurun_out/coopprof.txt 2>&1
rc=$?; tail -8 gpurun_out/coopprof.txt; exit $rc
