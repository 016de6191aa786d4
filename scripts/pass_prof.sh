# Phase profile of two read-only passes (a TCI_PASS_PROF=K variant, lib/variants/pprofK.so built by
# `make -C tensorcrossinterpolation.jl_amd/csrc variant NAME=pprofK VFLAGS=-DTCI_PASS_PROF=K`):
# the bench factorisation with the pass lines of pivots K and K + 1.   gpurun -- bash scripts/pass_prof.sh TAG K
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
T=${1:-pp}; K=${2:-27}
TCI_HIP_LIB=$PWD/tensorcrossinterpolation.jl_amd/lib/variants/pprof$K.so timeout -k 10 300 python -u bench.py --no-extras \
    --no-cpu --steps 1 --warmup 1 --epochs 3 > gpurun_out/${T}_pprof$K.log 2>&1 || { tail -20 gpurun_out/${T}_pprof$K.log; exit 1; }
grep "^\[pass\|^  \[k=" gpurun_out/${T}_pprof$K.log | head -40
