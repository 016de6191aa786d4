"""rocprof-based roofline of the rrLU read-only pass, from a rocprofv3 --kernel-trace --stats summary.

Usage: python scripts/trace_roofline.py KERNEL_STATS_CSV OUT_JSON [--m 8192 --n 8192 --r 256 --nb 10 --epochs 3]

Sorts the rrLU kernels of the traced bench command into families -- the initial argmax (k_pass2<0>,
one per factorisation, so it counts the factorisations), pass 0 (k_pass2<1,false,true>: reads A,
writes the shadow), the read-only passes (per-pass k_pass_mf<P,EXT,false> launches and the
persistent k_pass_mf_epoch launches, which run several passes each), refreshes, write-backs -- and
prices the read-only passes by the kernel trace alone: their total device time / the number of
read-only passes the schedule (bench.pass_bytes) gives per factorisation x the factorisations, against
the algorithmic bytes of those passes (--sh-bytes per trailing element: 1 for the 8-bit shadow of the
default build, 2 for fp16). This is
the rocprof counterpart of bench.py's HIP-event `roofline.frac`; bench.py reports it beside that one.
"""
import argparse
import csv
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def family(name):
    s = name.replace("void ", "").split("(")[0].strip()
    if s.startswith("tci::k_pass_mf_epoch<"):
        return "read_only_persistent"
    if s.startswith("tci::k_pass_mf<"):
        t = [x.strip() for x in s[s.index("<") + 1:s.rindex(">")].split(",")]
        return "refresh" if t[2] == "true" else "read_only_per_pass"
    if s.startswith("tci::k_pass_x<"):
        mode = s[s.index("<") + 1:s.rindex(">")].split(",")[0].strip()  # <MODE, NT>
        return {"1": "write_back", "2": "refresh"}.get(mode, "read_only_per_pass")
    if s.startswith("tci::k_pass2<"):
        t = [x.strip() for x in s[s.index("<") + 1:s.rindex(">")].split(",")]
        if t[0] == "0":
            return "initial_argmax"
        if t[1] == "true":
            return "write_back"
        if t[0] == "1" and t[2] == "true":
            return "pass0"
        return "read_only_per_pass"
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("stats")
    ap.add_argument("out")
    ap.add_argument("--m", type=int, default=8192)
    ap.add_argument("--n", type=int, default=8192)
    ap.add_argument("--r", type=int, default=256)
    ap.add_argument("--nb", type=int, default=10)
    ap.add_argument("--epochs", type=int, default=3)
    ap.add_argument("--sh-bytes", type=int, default=1)
    a = ap.parse_args()
    import bench
    fam = {}
    for row in csv.DictReader(open(a.stats)):
        f = family(row["Name"])
        if f is None:
            continue
        rec = fam.setdefault(f, {"launches": 0, "total_us": 0.0, "kernels": {}})
        rec["launches"] += int(row["Calls"])
        rec["total_us"] += float(row["TotalDurationNs"]) * 1e-3
        rec["kernels"][row["Name"].replace("void ", "").split("(")[0]] = {
            "calls": int(row["Calls"]), "avg_us": round(float(row["AverageNs"]) * 1e-3, 2)}
    nfact = fam.get("initial_argmax", {}).get("launches", 0)
    (ro_b, ro_n), (wb_b, wb_n), (rf_b, rf_n), (p0_b, p0_n) = bench.pass_bytes(
        a.m, a.n, a.r, a.nb, 1, True, a.sh_bytes, a.epochs, pass0_apart=True)
    ro_us = sum(fam.get(f, {}).get("total_us", 0.0) for f in ("read_only_per_pass", "read_only_persistent"))
    passes = ro_n * nfact
    out = {"source": os.path.relpath(a.stats), "config": vars(a), "factorisations": nfact, "families": fam}
    if passes:
        avg = ro_us / passes
        bpp = ro_b / ro_n
        out["read_only_pass"] = {
            "passes": passes, "avg_us_per_pass": round(avg, 3),
            "algorithmic_bytes_per_pass": bpp,
            "achieved_GBps": round(bpp / (avg * 1e-6) / 1e9, 1),
            "frac_of_8TBps": round(bpp / (avg * 1e-6) / 8e12, 4)}
    for f, (b, n_) in (("write_back", (wb_b, wb_n)), ("refresh", (rf_b, rf_n)), ("pass0", (p0_b, p0_n))):
        if f in fam and fam[f]["launches"]:
            avg = fam[f]["total_us"] / fam[f]["launches"]
            out[f] = {"avg_us": round(avg, 2), "algorithmic_bytes": b / max(n_, 1),
                      "achieved_GBps": round(b / max(n_, 1) / (avg * 1e-6) / 1e9, 1)}
    json.dump(out, open(a.out, "w"), indent=1)
    print(json.dumps({k: v for k, v in out.items() if k not in ("families",)}, indent=1))


if __name__ == "__main__":
    main()
