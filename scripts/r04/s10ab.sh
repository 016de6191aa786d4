# round-4 call 10a: A/B of the MFMA search's prologue ordering (pivot state first, map tests at
# their first use, branch-free pending-slot prefetch) against the HEAD build: bench + shapes
set -e
mkdir -p gpurun_out
T=r04s10a
V=$PWD/tensorcrossinterpolation.jl_amd/lib/variants
LIBS="default head" bash scripts/ab_lib.sh "TCI_RRLU_EPOCHS=3" > gpurun_out/${T}_ab.txt 2>&1 || { echo "ab rc=$?"; cat gpurun_out/${T}_ab.txt; exit 1; }
cat gpurun_out/${T}_ab.txt
for lib in default head; do
  if [ $lib = default ]; then unset TCI_HIP_LIB; else export TCI_HIP_LIB=$V/$lib.so; fi
  timeout -k 10 200 python -u scripts/ab_shapes.py --reps 7 --set 10,1 --set 10,3 --shape 2048x2048x256 --shape 4096x4096x256 --shape 8192x8192x256 > gpurun_out/${T}_shapes_$lib.jsonl 2>&1 || { echo "shapes $lib failed"; tail -5 gpurun_out/${T}_shapes_$lib.jsonl; exit 1; }
  echo "$lib"; python -c "
import json
for l in open('gpurun_out/${T}_shapes_$lib.jsonl'):
    try: d=json.loads(l)
    except Exception: continue
    print(d['m'], d['epochs'], d['ms_median'])"
done
echo done
