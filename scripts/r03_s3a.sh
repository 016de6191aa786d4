# round-3 session-3 start: GPU suite + smoke, default bench line, write-back A/B, small TCI2 configs
set -e
mkdir -p gpurun_out
T=r03s3a
timeout -k 10 400 python -u bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err
LIBS="default xs256" timeout -k 10 400 bash scripts/ab_lib.sh "AB=1" > gpurun_out/${T}_ab_xs.txt 2>&1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_gputest.txt 2>&1
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" >> gpurun_out/${T}_gputest.txt 2>&1
timeout -k 10 300 python -u scripts/tci2_configs.py C1_lorentz8d_parity C3_gauss20d C4_qosc40 C3_gaussmix20d C5_cp12d_K256 contract_mpo20 > gpurun_out/${T}_tci2.jsonl 2>&1
timeout -k 10 120 python -u scripts/small_abi_timing.py > gpurun_out/${T}_small_abi.jsonl 2>&1
echo done
