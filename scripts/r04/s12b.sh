# round-4 call 12b (s12 + s13 in one call while the pool is saturated): the grid-wide examination
# bound A/B'd against the HEAD build, then the full -m gpu suite (incl. config 5 as stated),
# smoke() and the full bench line of the final build
set -e
mkdir -p gpurun_out
T=r04s12b
LIBS="default head" bash scripts/ab_lib.sh "TCI_RRLU_EPOCHS=3" > gpurun_out/${T}_ab.txt 2>&1 || { echo "ab rc=$?"; cat gpurun_out/${T}_ab.txt; exit 1; }
cat gpurun_out/${T}_ab.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_gputest.txt 2>&1 || { echo "gputest rc=$?"; tail -30 gpurun_out/${T}_gputest.txt; exit 1; }
tail -2 gpurun_out/${T}_gputest.txt
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${T}_smoke.txt 2>&1 || { echo "smoke rc=$?"; tail -20 gpurun_out/${T}_smoke.txt; exit 1; }
tail -1 gpurun_out/${T}_smoke.txt
timeout -k 10 600 python -u bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { echo "bench rc=$?"; tail -20 gpurun_out/${T}_bench.err; exit 1; }
python -c "import json;d=json.loads(open('gpurun_out/${T}_bench.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'],json.dumps(d['roofline'])[:700]);print(json.dumps(d.get('cpu_baseline'))[:300])"
echo done
