# round-4 call 16: where the rrLU kernels' wave cycles go (one rocprofv3 --pmc pass of 8 SQ counters
# over the default bench command: waiting, issue-stalled, active, LDS stalls and bank conflicts,
# VALU), for the write-back and pass analysis in DESIGN
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_INSTS_VALU \
  --output-format csv -d "$R/gpurun_out/r04s16_sq" -o run -- python3 "$R/bench.py" --steps 2 --warmup 1 --no-extras --no-cpu > "$R/gpurun_out/r04s16_sq.log" 2>&1 || { echo "pmc rc=$?"; tail -20 "$R/gpurun_out/r04s16_sq.log"; exit 1; }
find "$R/gpurun_out/r04s16_sq" -name "*.csv"
echo done
