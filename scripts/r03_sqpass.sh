# SQ counters of the rrLU pass kernels (one --pmc pass, bench command): where the write-back
# pass (k_pass_x<1>) and the read-only passes spend their wave cycles
set -e
mkdir -p gpurun_out/r03_sq
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS --output-format csv -d gpurun_out/r03_sq/pmc1 -o run -- python3 bench.py --steps 2 --warmup 1 --no-extras --no-cpu > gpurun_out/r03_sq/pmc1.log 2>&1
python3 scripts/pmc_summary.py gpurun_out/r03_sq gpurun_out/r03_sq/summary.json > gpurun_out/r03_sq/summary.txt
echo done
