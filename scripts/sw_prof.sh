# Small-sweep (C3 / C4) evidence: the phase profile of the TCI_SW_PROF build (variants/swprof.so,
# built by `make -C tensorcrossinterpolation.jl_amd/csrc variant NAME=swprof VFLAGS=-DTCI_SW_PROF`),
# the host-side wall-time breakdown, and a kernel trace of the default build.
#   gpurun -- bash scripts/sw_prof.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
T=${1:-sw}
if [ -f tensorcrossinterpolation.jl_amd/lib/variants/swprof.so ]; then
  TCI_HIP_LIB=$PWD/tensorcrossinterpolation.jl_amd/lib/variants/swprof.so timeout -k 10 200 python -u scripts/tci2_configs.py C4_qosc40 C3_gauss20d > gpurun_out/${T}_swprof.log 2>&1 || { tail -20 gpurun_out/${T}_swprof.log; exit 1; }
  grep "sweep_small\] [0-9]\|wall_s" gpurun_out/${T}_swprof.log | cut -c1-300
fi
timeout -k 10 200 python -u scripts/small_breakdown.py > gpurun_out/${T}_breakdown.jsonl 2>&1 || { tail -20 gpurun_out/${T}_breakdown.jsonl; exit 1; }
cat gpurun_out/${T}_breakdown.jsonl
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
    -d $GRAFT_REPO_ROOT/gpurun_out/${T}_trace -o run -- python3 $GRAFT_REPO_ROOT/scripts/tci2_configs.py C4_qosc40 C3_gauss20d ) > gpurun_out/${T}_trace.log 2>&1 || { tail -20 gpurun_out/${T}_trace.log; exit 1; }
f=$(ls gpurun_out/${T}_trace/*/run_kernel_stats.csv 2>/dev/null | head -1); [ -z "$f" ] && f=$(ls gpurun_out/${T}_trace/run_kernel_stats.csv)
cut -d, -f1-6 "$f" | head -25
