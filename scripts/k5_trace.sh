# rocprofv3 kernel trace of the dense bench (K3 / K4 / K5) for one TCI_GETRF_NT setting: per-kernel
# times of the getrf panel chain.   gpurun -- bash scripts/k5_trace.sh TAG NT
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
T=${1:-k5t}; NT=${2:-256}
( cd /tmp && export TMPDIR=/tmp && export TCI_GETRF_NT=$NT && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv \
    -d $GRAFT_REPO_ROOT/gpurun_out/${T}_trace -o run -- python3 $GRAFT_REPO_ROOT/scripts/dense_bench.py ) \
    > gpurun_out/${T}_trace.log 2>&1 || { tail -20 gpurun_out/${T}_trace.log; exit 1; }
f=$(ls gpurun_out/${T}_trace/*/run_kernel_stats.csv 2>/dev/null | head -1); [ -z "$f" ] && f=$(ls gpurun_out/${T}_trace/run_kernel_stats.csv)
cut -d, -f1-4 "$f" | head -30
