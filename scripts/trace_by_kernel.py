"""Per-kernel-name duration summary of a rocprofv3 kernel trace csv (name truncated at '(')."""
import csv
import sys
from collections import defaultdict

d = defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    d[r["Kernel_Name"].split("(")[0].replace("void ", "")].append(
        (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-3)
for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1])):
    v.sort()
    print(f"{k[:44]:44s} n={len(v):5d} avg={sum(v) / len(v):9.2f}us med={v[len(v) // 2]:9.2f} "
          f"min={v[0]:9.2f} total={sum(v) / 1e3:8.2f}ms")
