"""fp64 VALU flops per Pi element of the quantics assembly from a rocprofv3 --pmc counter CSV:
python scripts/valu_summary.py run_counter_collection.csv out.json [elements_per_launch]
Wave-level instruction counts x 64 lanes; FMA = 2 flops, ADD / MUL / TRANS = 1."""
import csv
import json
import sys
from collections import defaultdict

path, out = sys.argv[1], sys.argv[2]
elems = float(sys.argv[3]) if len(sys.argv) > 3 else 8192.0 * 8192.0
tot = defaultdict(float)
disp = defaultdict(set)
for row in csv.DictReader(open(path)):
    name = row.get("Kernel_Name") or row.get("Kernel-Name") or ""
    if "k_assemble" not in name:
        continue
    cn = row.get("Counter_Name") or row.get("Counter-Name")
    tot[cn] += float(row.get("Counter_Value") or row.get("Counter-Value") or 0)
    disp[cn].add(row.get("Dispatch_Id") or row.get("Dispatch-Id"))
nl = max((len(v) for v in disp.values()), default=1)
w = {"SQ_INSTS_VALU_FMA_F64": 2.0, "SQ_INSTS_VALU_ADD_F64": 1.0, "SQ_INSTS_VALU_MUL_F64": 1.0,
     "SQ_INSTS_VALU_TRANS_F64": 1.0}
flops = sum(64.0 * w.get(k, 0.0) * v for k, v in tot.items())
res = {"counters_per_launch": {k: v / nl for k, v in tot.items()}, "launches": nl,
       "fp64_flops_per_element": flops / nl / elems,
       "note": "rocprofv3 --pmc SQ_INSTS_VALU_{FMA,ADD,MUL,TRANS}_F64 over k_assemble<QOSC>; x 64 lanes"}
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res))
