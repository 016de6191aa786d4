"""Repeatability of a TCI2 sweep: runs a config several times in one process and reports whether
ranks, errors and pivot sets are identical.   python scripts/tci2_repeat.py [K] [maxbonddim] [reps]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tensorcrossinterpolation.jl_amd"))

import numpy as np  # noqa: E402

import tci_amd as T  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 256
mb = int(sys.argv[2]) if len(sys.argv) > 2 else 256
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
rng = np.random.default_rng(2)
L, d = 12, 32
f = T.cp_function(0.5 + rng.random((K, L, d)))
p0 = T.optfirstpivot(f, [d] * L)
out = []
for r in range(reps):
    tci, ranks, errors = T.crossinterpolate2(f, [d] * L, [p0], tolerance=1e-10, maxbonddim=mb, maxiter=3,
                                             nsearchglobalpivot=0)
    out.append((ranks, errors, [np.asarray(s).copy() for s in tci.Iset], [np.asarray(s).copy() for s in tci.Jset],
                tci.maxsamplevalue))
    print(r, ranks, [float(e) for e in errors], "maxsample", tci.maxsamplevalue, flush=True)
for r in range(1, reps):
    a, b = out[0], out[r]
    same_sets = all(np.array_equal(x, y) for x, y in zip(a[2] + a[3], b[2] + b[3]))
    print(f"run {r} vs 0: ranks {a[0] == b[0]} errors {a[1] == b[1]} sets {same_sets}")
