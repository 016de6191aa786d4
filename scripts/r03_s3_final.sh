# round-3 session-3 final evidence on one MI355X: GPU suite + smoke, default bench line (with extras: K5 register panel), kernel trace + PMC
# passes of the bench command, TCI2 configs (C5 at full scale included)
set -e
mkdir -p gpurun_out
T=r03s3z
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_gputest.txt 2>&1
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" >> gpurun_out/${T}_gputest.txt 2>&1
timeout -k 10 400 python -u bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err
bash scripts/profile_round.sh gpurun_out/prof_${T} > gpurun_out/${T}_prof.log 2>&1
timeout -k 10 300 python -u scripts/tci2_configs.py C1_lorentz8d_parity C3_gauss20d C4_qosc40 C3_gaussmix20d C5_cp12d_K256 contract_mpo20 > gpurun_out/${T}_tci2.jsonl 2>&1
timeout -k 10 300 python -u scripts/tci2_configs.py C5_cp12d_K1024 >> gpurun_out/${T}_tci2.jsonl 2>&1
echo done
