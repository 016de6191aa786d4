"""Where the rrLU kernels' wave cycles go: one rocprofv3 --pmc pass of SQ counters
(scripts/r04/s16.sh) summarised per kernel family (scripts/pmc_summary.py's families).

Usage: python scripts/sq_breakdown.py PMC_DIR [OUT_JSON]

SQ_WAVE_CYCLES = SQ_WAIT_ANY (parked on s_waitcnt / barrier) + SQ_WAIT_INST_ANY (issue-stalled)
+ SQ_ACTIVE_INST_ANY (issuing), all in quad-cycles (MI355X_MICROARCH.md "rocprofv3 PMC slots");
SQ_WAIT_INST_LDS is the LDS share of the issue stalls, SQ_ACTIVE_INST_VALU the VALU share of the
issuing cycles. Fractions are of SQ_WAVE_CYCLES, summed over the dispatches of a family.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import family  # noqa: E402


def summarise(root):
    tot = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    for f in sorted(glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True)):
        for row in csv.DictReader(open(f)):
            fam = family(row["Kernel_Name"])
            tot[fam][row["Counter_Name"]] += float(row["Counter_Value"])
            disp[fam].add((f, row["Dispatch_Id"]))
    out = {}
    for fam, d in tot.items():
        w = d.get("SQ_WAVE_CYCLES", 0.0)
        rec = {"dispatches": len(disp[fam])}
        rec.update({c: v / len(disp[fam]) for c, v in sorted(d.items())})
        if w > 0:
            for c, key in (("SQ_WAIT_ANY", "frac_waiting"), ("SQ_WAIT_INST_ANY", "frac_issue_stalled"),
                           ("SQ_ACTIVE_INST_ANY", "frac_issuing"), ("SQ_WAIT_INST_LDS", "frac_lds_stalled"),
                           ("SQ_ACTIVE_INST_VALU", "frac_valu")):
                if c in d:
                    rec[key] = round(d[c] / w, 4)
        out[fam] = rec
    return out


if __name__ == "__main__":
    res = summarise(sys.argv[1])
    if len(sys.argv) > 2:
        with open(sys.argv[2], "w") as fh:
            json.dump(res, fh, indent=1, sort_keys=True)
    for fam, rec in sorted(res.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0) * kv[1]["dispatches"]):
        print(f"{fam[:44]:44s} n={rec['dispatches']:5d} wait={rec.get('frac_waiting', float('nan')):.3f} "
              f"stall={rec.get('frac_issue_stalled', float('nan')):.3f} issue={rec.get('frac_issuing', float('nan')):.3f} "
              f"lds_stall={rec.get('frac_lds_stalled', float('nan')):.3f} valu={rec.get('frac_valu', float('nan')):.3f} "
              f"bank_conf={rec.get('SQ_LDS_BANK_CONFLICT', float('nan')):.3g}")
