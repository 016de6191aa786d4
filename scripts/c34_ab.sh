# C3 / C4 end-to-end wall time with the one-wave small-sweep rrLU off / on (TCI_SW_LUWAVE)
set -o pipefail
cd $GRAFT_REPO_ROOT
for v in 0 1 0 1; do
  echo "TCI_SW_LUWAVE=$v"
  TCI_SW_LUWAVE=$v timeout -k 10 300 python -u scripts/tci2_configs.py C3_gauss20d C4_qosc40 || exit 1
done
