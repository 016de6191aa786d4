"""Summary of the [census ...] lines of a census build's run (scripts/exam_census.sh): per log, the
factorisations' read-only passes (flush=0) with exact examinations over the grid -- mean, median,
max, the pass with the most -- and the certificate failures counted by the last pass."""
import json
import re
import sys

out = {}
for path in sys.argv[1:]:
    runs, cur = [], []
    for ln in open(path):
        m = re.match(r"\[census k=(\d+) P=(\d+) flush=(\d+) grid=(\d+)\] exams (\d+) cert_fails (\d+)", ln)
        if not m:
            continue
        k, P, fl, grid, ex, cf = map(int, m.groups())
        if k == 0 and cur:  # the initial argmax starts a factorisation
            runs.append(cur)
            cur = []
        cur.append((k, P, fl, ex, cf))
    if cur:
        runs.append(cur)
    recs = []
    for r in runs:
        ro = [(k, ex) for (k, P, fl, ex, cf) in r if not fl and k >= 2]  # k 0 / 1: initial argmax / pass 0 (exact)
        if not ro:
            continue
        xs = sorted(ex for _, ex in ro)
        kmax = max(ro, key=lambda t: t[1])
        recs.append({"passes": len(ro), "exams_mean": round(sum(xs) / len(xs), 1), "exams_median": xs[len(xs) // 2],
                     "exams_max": kmax[1], "exams_max_at_k": kmax[0], "exams_total": sum(xs),
                     "cert_fails": r[-1][4] - r[0][4]})
    out[path] = recs[-1] if recs else None
print(json.dumps(out, indent=1))
