# round-3 full check on one MI355X: GPU suite + smoke, default bench line, TCI2 small/large configs
# usage (from the repo root on the GPU box): bash scripts/r03_full.sh TAG
set -e
T=${1:-r03}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_gputest.txt 2>&1
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" >> gpurun_out/${T}_gputest.txt 2>&1
timeout -k 10 400 python -u bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err
timeout -k 10 300 python -u scripts/tci2_configs.py C1_lorentz8d_parity C3_gauss20d C4_qosc40 C3_gaussmix20d C5_cp12d_K256 > gpurun_out/${T}_tci2_small.jsonl 2>&1
echo done
