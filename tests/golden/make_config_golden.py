"""Golden TCI2 results for the BASELINE configurations (scaled where the full size would take the
CPU oracle minutes), produced by the oracle (pinned by the reference's known-answer tests; the
reference itself is Julia and cannot run here). Writes tests/golden/config_golden.json.

  python tests/golden/make_config_golden.py [name ...]   (only the named configs are re-made;
                                                      the others are kept from the JSON)
Configs marked "cpu_check": False take the 1-core oracle many minutes (C5 at CP rank 256: Pi of
9216 x 9216, rrLU at r = 256 on the pass pipeline with two staging groups); the CPU suite does not
re-derive them, the GPU suite checks the product against them.
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))

import oracle_lib as O  # noqa: E402

QOSC = [10.0, 2 * np.pi * 100, 1.1]


def configs():
    rng = np.random.default_rng(3)
    centres = rng.uniform(1, 8, (8, 8))
    gm = np.concatenate([[8, 0.05], centres.ravel(), np.ones(8)]).tolist()
    g = 0.5 + np.random.default_rng(2).random((16, 6, 8))
    cp = np.concatenate([[16, 8], g.ravel()]).tolist()
    g256 = 0.5 + np.random.default_rng(6).random((256, 8, 36))
    cp256 = np.concatenate([[256, 36], g256.ravel()]).tolist()
    # Contraction(A, B) of two 5-site MPOs (contraction.jl:60; TCI_F_MPO params, see
    # tci_amd.contraction._mpo_params): bonds [1,3,4,4,3,1], d1 = d2 = d3 = 2
    mrng = np.random.default_rng(4)
    bonds = [1, 3, 4, 4, 3, 1]
    A = [mrng.standard_normal((bonds[n], 2, 2, bonds[n + 1])) for n in range(5)]
    B = [mrng.standard_normal((bonds[n], 2, 2, bonds[n + 1])) for n in range(5)]
    hdr, blob, off = [5], [], 0
    for a, b in zip(A, B):
        hdr += [a.shape[0], 2, 2, a.shape[3], b.shape[0], 2, b.shape[3], off, off + a.size]
        blob += a.ravel(order="F").tolist() + b.ravel(order="F").tolist()
        off += a.size + b.size
    mpo = [float(x) for x in hdr] + blob
    return [
        {"name": "C1_lorentz8d", "kind": 1, "params": [1.0], "localdims": [10] * 8, "initialpivots": None,
         "kw": {"tolerance": 1e-8}},
        {"name": "C3_gauss20d_d16", "kind": 3, "params": [0.05, 8.5], "localdims": [16] * 20,
         "initialpivots": [[8] * 20], "kw": {"tolerance": 1e-10, "maxbonddim": 512}},
        {"name": "C3p_gaussmix8d_K8", "kind": 4, "params": gm, "localdims": [8] * 8,
         "initialpivots": [[int(round(c)) for c in centres[0]]], "kw": {"tolerance": 1e-10}},
        {"name": "C4_qosc40", "kind": 5, "params": QOSC, "localdims": [2] * 40,
         "initialpivots": [[1] + [2] * 39], "kw": {"tolerance": 1e-8}},
        {"name": "C5_cp6d_K16", "kind": 8, "params": cp, "localdims": [8] * 6, "initialpivots": [[1] * 6],
         "kw": {"tolerance": 1e-10}},
        # config 5 at CP rank 256 (SURVEY 8(d) C5 scaled): 8 legs of d = 36, so the second
        # iteration's Pi are (256 * 36)^2 = 9216^2 -- 18 row tiles of the pass pipeline, two staging
        # groups -- factorised to r = 256 (C5's only fixture stayed in k_rrlu_small)
        {"name": "C5_cp8d_d36_K256", "kind": 8, "params": cp256, "localdims": [36] * 8,
         "initialpivots": [[1] * 8], "kw": {"tolerance": 1e-10, "maxbonddim": 256, "maxiter": 2},
         "cpu_check": False},
        {"name": "contract_mpo5", "kind": 9, "params": mpo, "localdims": [4] * 5, "initialpivots": [[1] * 5],
         "kw": {"tolerance": 1e-12}},
    ]


def run(c):
    t, ranks, errors = O.crossinterpolate2(c["kind"], c["params"], c["localdims"], c["initialpivots"], **c["kw"])
    L = len(c["localdims"])
    rng = np.random.default_rng(0)
    X = np.stack([rng.integers(1, d + 1, 64) for d in c["localdims"]], axis=1).astype(np.int32)
    return {"ranks": [int(r) for r in ranks], "errors": [float(e) for e in errors],
            "linkdims": t.linkdims(), "maxsamplevalue": t.maxsamplevalue,
            "Iset": [t.Iset(p).tolist() for p in range(L)], "Jset": [t.Jset(p).tolist() for p in range(L)],
            "points": X.tolist(), "values": [t.evaluate(x) for x in X]}


if __name__ == "__main__":
    path = os.path.join(HERE, "config_golden.json")
    old = {c["name"]: c for c in json.load(open(path))} if os.path.exists(path) else {}
    only = set(sys.argv[1:])
    out = []
    for c in configs():
        if only and c["name"] not in only and c["name"] in old:
            out.append(old[c["name"]])
            continue
        r = run(c)
        print(c["name"], r["ranks"], r["errors"][-1], flush=True)
        out.append({**c, "result": r})
    with open(path, "w") as fh:
        json.dump(out, fh)
