# SQ counters of the device-resident sweep kernel (instruction fetch / wait vs issue)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_IFETCH SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_ANY -d gpurun_out/r03_sq -o sq -- python3 scripts/small_breakdown.py > gpurun_out/r03_sq.log 2>&1
