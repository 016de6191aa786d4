# rocprofv3 kernel trace of config 5 as stated (scripts/tci2_configs.py C5_cp12d_K1024): where the
# ~25 s of device time go, by kernel.   gpurun -- bash scripts/c5_trace.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
T=${1:-c5}
( cd /tmp && export TMPDIR=/tmp && timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv \
    -d $GRAFT_REPO_ROOT/gpurun_out/${T}_trace -o run -- python3 $GRAFT_REPO_ROOT/scripts/tci2_configs.py C5_cp12d_K1024 ) \
    > gpurun_out/${T}_trace.log 2>&1 || { tail -20 gpurun_out/${T}_trace.log; exit 1; }
f=$(ls gpurun_out/${T}_trace/*/run_kernel_stats.csv 2>/dev/null | head -1); [ -z "$f" ] && f=$(ls gpurun_out/${T}_trace/run_kernel_stats.csv)
cut -d, -f1-5 "$f" | head -30
grep wall_s gpurun_out/${T}_trace.log | cut -c1-300
