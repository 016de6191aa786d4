"""Summarise rocprofv3 PMC csv passes per kernel family (mean per dispatch)."""
import csv
import glob
import os
import sys
from collections import defaultdict

root = sys.argv[1]
agg = defaultdict(lambda: defaultdict(list))
durs = defaultdict(list)
for f in sorted(glob.glob(os.path.join(root, "pmc*", "run_counter_collection.csv"))):
    for row in csv.DictReader(open(f)):
        name = row["Kernel_Name"]
        short = name.split("(")[0].replace("void ", "")
        if "k_pass" in short:
            short = short + ("" if "true" not in short else "")
        agg[short][row["Counter_Name"]].append(float(row["Counter_Value"]))
        agg[short]["_vgpr"].append(float(row["VGPR_Count"]))
        durs[short].append((int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) * 1e-3)
for k in sorted(agg, key=lambda k: -sum(durs[k])):
    d = agg[k]
    line = f"{k[:60]:60s} n={len(durs[k]) // max(1, len([c for c in d if c != '_vgpr'])):4d} us={sum(durs[k]) / len(durs[k]):8.1f}"
    for c in sorted(d):
        v = sum(d[c]) / len(d[c])
        line += f" {c}={v:.4g}"
    print(line)
