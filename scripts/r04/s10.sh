# round-4 call 10: rocprofv3 kernel trace + PMC passes of the default bench command on the built
# commit (scripts/profile_round.sh), then the full bench line with extras
set -e
mkdir -p gpurun_out
T=r04s10
timeout -k 10 900 bash scripts/profile_round.sh gpurun_out/${T}_prof > gpurun_out/${T}_prof.log 2>&1 || { echo "profile rc=$?"; tail -20 gpurun_out/${T}_prof.log; exit 1; }
tail -3 gpurun_out/${T}_prof.log
timeout -k 10 900 python -u bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { echo "bench rc=$?"; tail -20 gpurun_out/${T}_bench.err; exit 1; }
python -c "import json;d=json.loads(open('gpurun_out/${T}_bench.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'],json.dumps(d['roofline'])[:600]);print(json.dumps(d.get('cpu_baseline'))[:300])"
echo done
