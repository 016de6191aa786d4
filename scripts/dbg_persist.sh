# diagnostic call: the persistent epoch launch against the per-pass launches and the oracle
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for mp in 2 3 9; do TCI_EPOCH_MAXPASS=$mp timeout -k 10 120 python -u scripts/persist_debug.py 2100 1900 40 10 1 || exit 1; done
TCI_RRLU_SERP=0 timeout -k 10 120 python -u scripts/persist_debug.py 2100 1900 40 10 1 || exit 1
