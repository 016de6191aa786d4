"""Summarise rocprofv3 PMC passes (scripts/profile_round.sh) per kernel family.

Usage: python scripts/pmc_summary.py PMC_DIR [OUT_JSON]

Every pmc*/ directory under PMC_DIR holds one counter group's run_counter_collection.csv. Values
are averaged per dispatch. FETCH_SIZE / WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE counts half
the bytes of a wide coalesced streaming read (MI355X_MICROARCH.md "HBM"), so read bytes =
2 x FETCH_SIZE x 1024. The stream-read kernel of the same run (k_stream_read, a known byte count)
is kept in the summary as the calibration check of that factor.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def family(name):
    short = name.split("(")[0].replace("void ", "").strip()
    if short.startswith("tci::k_pass_mf_epoch<"):  # persistent shadow-epoch launch (several passes each)
        return "rrlu_read_only_persistent"
    if short.startswith("tci::k_pass_mf<"):  # <P, EXT, RF>: RF = the shadow refresh pass
        targs = [t.strip() for t in short[short.index("<") + 1:short.rindex(">")].split(",")]
        return "rrlu_refresh_pass" if len(targs) > 2 and targs[2] == "true" else "rrlu_read_only_pass"
    if short.startswith("tci::k_pass_sh<"):
        return "rrlu_read_only_pass"
    if short.startswith("tci::k_pass_x<"):  # <MODE>: 1 write-back, 0 / 2 exact fallbacks
        mode = short[short.index("<") + 1:short.rindex(">")].split(",")[0].strip()  # <MODE, NT>
        return {"1": "rrlu_write_back_pass", "2": "rrlu_refresh_pass"}.get(mode, "rrlu_read_only_pass")
    if short.startswith(("tci::k_pass<", "tci::k_pass2<")):
        targs = [t.strip() for t in short[short.index("<") + 1:short.rindex(">")].split(",")]
        if targs[1] == "true":
            return "rrlu_write_back_pass"
        if targs[0] == "0":  # the initial argmax of A (k = -1)
            return "rrlu_initial_pass"
        if targs[0] == "1" and len(targs) > 2 and targs[2] == "true":  # pass 0: reads A, writes the shadow
            return "rrlu_pass0"
        return "rrlu_read_only_pass"
    return short


def summarise(root):
    vals = defaultdict(lambda: defaultdict(list))
    durs = defaultdict(list)
    for f in sorted(glob.glob(os.path.join(root, "pmc*", "**", "*counter_collection.csv"), recursive=True)):
        seen = set()
        for row in csv.DictReader(open(f)):
            fam = family(row["Kernel_Name"])
            vals[fam][row["Counter_Name"]].append(float(row["Counter_Value"]))
            key = (f, row["Dispatch_Id"])
            if key not in seen:
                seen.add(key)
                durs[fam].append((int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) * 1e-3)
    out = {}
    for fam, d in vals.items():
        rec = {"dispatches_profiled": len(durs[fam]),
               "avg_us_under_pmc": round(sum(durs[fam]) / max(len(durs[fam]), 1), 2)}
        for c, v in sorted(d.items()):
            rec[c] = sum(v) / len(v)
        if "FETCH_SIZE" in rec:
            rec["read_bytes_per_launch"] = 2.0 * rec["FETCH_SIZE"] * 1024.0
        if "WRITE_SIZE" in rec:
            rec["write_bytes_per_launch"] = rec["WRITE_SIZE"] * 1024.0
        if "read_bytes_per_launch" in rec and "write_bytes_per_launch" in rec:
            rec["hbm_bytes_per_launch"] = rec["read_bytes_per_launch"] + rec["write_bytes_per_launch"]
        out[fam] = rec
    return out


if __name__ == "__main__":
    res = summarise(sys.argv[1])
    if len(sys.argv) > 2:
        with open(sys.argv[2], "w") as fh:
            json.dump(res, fh, indent=1, sort_keys=True)
    for fam, rec in sorted(res.items(), key=lambda kv: -kv[1]["avg_us_under_pmc"] * kv[1]["dispatches_profiled"]):
        print(f"{fam[:48]:48s} n={rec['dispatches_profiled']:5d} us={rec['avg_us_under_pmc']:9.2f} "
              f"read={rec.get('read_bytes_per_launch', float('nan')) / 1e6:9.2f}MB "
              f"write={rec.get('write_bytes_per_launch', float('nan')) / 1e6:9.2f}MB")
