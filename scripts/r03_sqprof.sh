# SQ / SQC counters of the device-resident sweep kernel: instruction-cache behaviour (one pass)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_VALU -d gpurun_out/r03_sqc -o sq -- python3 scripts/small_breakdown.py > gpurun_out/r03_sqc.log 2>&1
