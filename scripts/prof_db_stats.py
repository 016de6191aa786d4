"""Kernel summary (name, calls, total/avg ns) from a rocprofv3 SQLite results database, as CSV
like --stats' kernel_stats.csv: python scripts/prof_db_stats.py run_results.db [out.csv]"""
import csv
import sqlite3
import sys

db = sqlite3.connect(sys.argv[1])
cols = [r[1] for r in db.execute("pragma table_info(kernels)")]
name_col = "name" if "name" in cols else ("kernel_name" if "kernel_name" in cols else None)
rows = db.execute(f"select {name_col}, count(*), sum(end - start), avg(end - start), min(end - start), "
                  f"max(end - start) from kernels group by {name_col} order by sum(end - start) desc").fetchall()
tot = sum(r[2] for r in rows) or 1
out = open(sys.argv[2], "w", newline="") if len(sys.argv) > 2 else sys.stdout
w = csv.writer(out)
w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
for r in rows:
    w.writerow([r[0], r[1], r[2], round(r[3], 1), round(100.0 * r[2] / tot, 2), r[4], r[5]])
