set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for k in 3 1 2; do TCI_EPOCH_KINDS=$k timeout -k 10 120 python -u scripts/persist_debug.py 2100 1900 150 10 3 || exit 1; done
TCI_EPOCH_KINDS=3 timeout -k 10 120 python -u scripts/persist_debug.py 2100 1900 150 10 1 || exit 1
