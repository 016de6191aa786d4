#!/bin/bash
# One gpurun call = one invocation of this driver with a list of steps, run from the repository
# root on the GPU box:
#   gpurun --timeout 1200 -- bash scripts/gpucall.sh TAG step [step ...]
# Every step writes under gpurun_out/TAG_*, runs under its own time limit, and the first failing
# step ends the call (no GPU step runs after a failure). Steps:
#   tests[:EXPR]       python -m pytest tests -m gpu [-k EXPR]                 -> TAG_gputest.txt
#   smoke              __graft_entry__.smoke()                                  -> TAG_smoke.txt
#   bench[:ARGS]       python bench.py ARGS (default: the driver's command)      -> TAG_bench.json
#   ab:LIBS:CFGS       A/B of library variants x env settings (scripts/ab_lib.sh; LIBS and CFGS
#                      comma-separated, e.g. ab:default,persist:TCI_RRLU_PERSIST=0,TCI_RRLU_PERSIST=1)
#   trace[:ARGS]       rocprofv3 --kernel-trace --stats of bench.py ARGS       -> TAG_trace/
#   pmc:C1+C2[:ARGS]   one rocprofv3 --pmc pass of counters C1 C2 ... over bench.py ARGS -> TAG_pmcN/
#   pmcsum             scripts/pmc_summary.py over this call's TAG_pmc* passes -> TAG_pmc_summary.json
#   avail              rocprofv3 --list-avail                                  -> TAG_avail.txt
#   py:SCRIPT[:ARGS]   python SCRIPT ARGS                                      -> TAG_py_SCRIPT.txt
# Round 4's one-off call scripts (scripts/r04/sN.sh) are in the git history; what each ran, and
# which profiles/ files each call's results became, is listed in profiles/README.md.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
TAG=$1; shift
O=gpurun_out/$TAG
BENCH_DEFAULT="--steps 3 --warmup 1 --no-extras --no-cpu"
npmc=0
fail() { echo "[$TAG] step '$1' failed (rc $2)"; [ -f "$3" ] && tail -30 "$3"; exit 1; }
for step in "$@"; do
  name=${step%%:*}; arg=""; [ "$name" != "$step" ] && arg=${step#*:}
  echo "[$TAG] step $step ($(date +%T))"
  case $name in
    tests)
      k=(); [ -n "$arg" ] && k=(-k "$arg")
      timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread "${k[@]}" \
        > ${O}_gputest.txt 2>&1 || fail "$step" $? ${O}_gputest.txt
      tail -2 ${O}_gputest.txt ;;
    smoke)
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > ${O}_smoke.txt 2>&1 \
        || fail "$step" $? ${O}_smoke.txt
      tail -1 ${O}_smoke.txt ;;
    bench)
      timeout -k 10 600 python -u bench.py ${arg} > ${O}_bench.json 2> ${O}_bench.err || fail "$step" $? ${O}_bench.err
      tail -c 400 ${O}_bench.json; echo ;;
    ab)
      libs=${arg%%:*}; cfgs=${arg#*:}
      IFS=, read -ra CF <<< "$cfgs"
      LIBS="${libs//,/ }" timeout -k 10 900 bash scripts/ab_lib.sh "${CF[@]}" > ${O}_ab.txt 2>&1 || fail "$step" $? ${O}_ab.txt
      cat ${O}_ab.txt ;;
    trace)
      ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv \
          -d "$R/${O}_trace" -o run -- python3 "$R/bench.py" ${arg:-$BENCH_DEFAULT} ) > ${O}_trace.log 2>&1 \
        || fail "$step" $? ${O}_trace.log
      tail -c 300 ${O}_trace.log; echo ;;
    pmc)
      npmc=$((npmc + 1))
      ctrs=${arg%%:*}; bargs=""; [ "$ctrs" != "$arg" ] && bargs=${arg#*:}
      ( cd /tmp && export TMPDIR=/tmp && timeout -s KILL 300 rocprofv3 --pmc ${ctrs//+/ } --output-format csv \
          -d "$R/${O}_pmc$npmc" -o run -- python3 "$R/bench.py" ${bargs:-$BENCH_DEFAULT} ) > ${O}_pmc$npmc.log 2>&1 \
        || fail "$step" $? ${O}_pmc$npmc.log
      echo "pmc pass $npmc ($ctrs) ok" ;;
    pmcsum)
      mkdir -p ${O}_pmcall && for d in ${O}_pmc[0-9]*; do [ -d "$d" ] && ln -sfn "$R/$d" ${O}_pmcall/$(basename $d | sed "s/^${TAG}_//"); done
      python scripts/pmc_summary.py ${O}_pmcall ${O}_pmc_summary.json > ${O}_pmcsum.txt 2>&1 || fail "$step" $? ${O}_pmcsum.txt
      echo "pmc summary -> ${O}_pmc_summary.json" ;;
    avail)
      ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 120 rocprofv3 --list-avail ) > ${O}_avail.txt 2>&1 || fail "$step" $? ${O}_avail.txt
      grep -c . ${O}_avail.txt ;;
    py)
      script=${arg%%:*}; pargs=""; [ "$script" != "$arg" ] && pargs=${arg#*:}
      timeout -k 10 900 python -u $script ${pargs//,/ } > ${O}_py_$(basename $script .py).txt 2>&1 \
        || fail "$step" $? ${O}_py_$(basename $script .py).txt
      tail -5 ${O}_py_$(basename $script .py).txt ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "[$TAG] done ($(date +%T))"
