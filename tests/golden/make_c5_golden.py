"""Golden TCI2 result for config 5 AS STATED (BASELINE.json configs[4]): 12 legs of d = 32, the
CP-rank-1024 synthetic of SURVEY 8(d), tolerance 1e-10, maxbonddim 1024, maxiter 3,
nsearchglobalpivot = 0. Writes tests/golden/c5_golden.json. TEST INFRASTRUCTURE ONLY.

The oracle runs in its fast mode (oracle/tci_oracle.c "fast mode": the OpenMP rrLU, bitwise equal to
the loop-for-loop one; CP evaluated factorised at the bond; the site-tensor solves, which are never
read in deterministic mode, skipped). Even so its 28 rrLUs of 32768^2 at r = 1024 take the CPU of a
GPU box's host about a minute each, so optimize! (tensorci2.jl:1018-1172, restated below exactly as
orc_tci_optimize does it) is split into half-sweeps with a checkpoint after each (orc_tci_save: the
index sets, the last history entry, pivot / bond errors, maxsamplevalue -- everything the next
half-sweep reads) and the per-iteration abstol kept beside it, so the run can span several calls:

  python tests/golden/make_c5_golden.py --state oracle/_ckpt/c5 [--halves N] [--threads T]

runs at most N more half-sweeps (default: all), then, once every iteration is done, the final
sweep1site! and the outputs (ranks, errors, link dims, index sets, 64 sampled values). The command
lines used for the committed fixture are recorded in its "provenance" field.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))

K, L, D = 1024, 12, 32
TOL, MAXBOND, MAXITER = 1e-10, 1024, 3
NCHECK = 3


def params():
    g = 0.5 + np.random.default_rng(2).random((K, L, D))  # as scripts/tci2_configs.py cp12_full
    return np.concatenate([[K, D], g.ravel()])


def optfirstpivot(O, p, localdims, maxsweep=1000):
    """optfirstpivot (util.jl:260-298) on the oracle's f, sequential as written."""
    n = len(localdims)
    pivot = [1] * n
    ld = list(localdims)
    valf = abs(O.feval(8, p, ld, pivot))
    for _ in range(maxsweep):
        prev = valf
        for i in range(n):
            for d in range(1, localdims[i] + 1):
                x = list(pivot)
                x[i] = d
                v = abs(O.feval(8, p, ld, x))
                if v > valf:
                    valf = v
                    pivot[i] = d
        if prev == valf:
            break
    return pivot


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--state", required=True)
    ap.add_argument("--halves", type=int, default=1 << 30)
    ap.add_argument("--threads", type=int, default=0)
    a = ap.parse_args()
    if a.threads:
        os.environ["OMP_NUM_THREADS"] = str(a.threads)
    import oracle_lib as O

    os.makedirs(a.state, exist_ok=True)
    prog_path = os.path.join(a.state, "progress.json")
    ckpt = os.path.join(a.state, "tci.ckpt")
    p = params()
    ld = [D] * L
    if os.path.exists(prog_path):
        prog = json.load(open(prog_path))
    else:
        p0 = optfirstpivot(O, p, ld)
        prog = {"p0": p0, "halves": 0, "abstol": [], "ranks": [], "errors": [], "done": False,
                "log": []}
    t = O.OracleTCI2(8, p, ld, [prog["p0"]], fast=True)
    if prog["halves"] > 0:
        t.load(ckpt)
    ran = 0
    while not prog["done"] and ran < a.halves:
        h = prog["halves"]
        it = h // 2 + 1  # outer iteration (1-based), tensorci2.jl:1088
        if h % 2 == 0:
            prog["abstol"].append(TOL * t.maxsamplevalue)  # :1089-1090 (normalizeerror)
        abstol = prog["abstol"][it - 1]
        t0 = time.time()
        # sweep2site!(tci, f, 2; ...) split into its two half-sweeps; fillsitetensors! after both
        t.sweep2site(niter=1, iter1=1 + h % 2, abstol=abstol, maxbonddim=MAXBOND,
                     fillsitetensors=(h % 2 == 1))
        prog["halves"] = h + 1
        prog["log"].append({"half": h + 1, "seconds": round(time.time() - t0, 1),
                            "linkdims": t.linkdims()})
        if h % 2 == 1:
            prog["errors"].append(float(t.pivoterror()))  # maxbonderror (:1118)
            prog["ranks"].append(int(t.rank()))
            n = len(prog["ranks"])
            conv = O.convergencecriterion(prog["ranks"], prog["errors"], [0] * n, abstol, MAXBOND, NCHECK)
            if conv or n >= MAXITER:
                prog["done"] = True
        t.save(ckpt)
        json.dump(prog, open(prog_path, "w"))
        print(json.dumps(prog["log"][-1]), flush=True)
        ran += 1
    if not prog["done"]:
        print("state saved after", prog["halves"], "half-sweeps", flush=True)
        return
    # final sweep1site! (:1160-1167) and errors ./ errornormalization (:1171)
    t0 = time.time()
    errnorm = t.maxsamplevalue
    t.sweep1site(True, 1e-14, TOL * errnorm, MAXBOND, True)
    rng = np.random.default_rng(0)
    X = np.stack([rng.integers(1, d + 1, 64) for d in ld], axis=1).astype(np.int32)
    res = {"ranks": prog["ranks"], "errors": [e / errnorm for e in prog["errors"]],
           "linkdims": t.linkdims(), "maxsamplevalue": t.maxsamplevalue,
           "Iset": [t.Iset(q).tolist() for q in range(L)], "Jset": [t.Jset(q).tolist() for q in range(L)],
           "points": X.tolist(), "values": [t.evaluate(x) for x in X]}
    out = {"name": "C5_cp12d_K1024_as_stated", "kind": 8, "K": K, "L": L, "d": D,
           "params_rng": "0.5 + numpy.random.default_rng(2).random((1024, 12, 32))",
           "initialpivots": [prog["p0"]],
           "kw": {"tolerance": TOL, "maxbonddim": MAXBOND, "maxiter": MAXITER},
           "oracle": "liboracle_fast.so (tci_oracle.c fast mode)",
           "half_sweep_log": prog["log"] + [{"sweep1site_and_outputs_s": round(time.time() - t0, 1)}],
           "result": res}
    json.dump(out, open(os.path.join(HERE, "c5_golden.json"), "w"))
    print("wrote c5_golden.json", res["ranks"], res["errors"], flush=True)


if __name__ == "__main__":
    main()
