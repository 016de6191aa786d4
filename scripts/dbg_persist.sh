# diagnostic call: the persistent epoch launch against the per-pass launches and the oracle
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for ep in 3 1; do timeout -k 10 120 python -u scripts/persist_debug.py 2100 1900 150 10 $ep || exit 1; done
