# round-4 call 18: the committed default build (deep write-back drain on): the whole -m gpu suite,
# smoke() and the default bench line
set -e
mkdir -p gpurun_out
T=r04s18
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_gputest.txt 2>&1 || { echo "gputest rc=$?"; tail -30 gpurun_out/${T}_gputest.txt; exit 1; }
tail -2 gpurun_out/${T}_gputest.txt
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${T}_smoke.txt 2>&1 || { echo "smoke rc=$?"; tail -20 gpurun_out/${T}_smoke.txt; exit 1; }
tail -1 gpurun_out/${T}_smoke.txt
timeout -k 10 600 python -u bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { echo "bench rc=$?"; tail -20 gpurun_out/${T}_bench.err; exit 1; }
tail -c 600 gpurun_out/${T}_bench.json
echo done
