"""Repeatability of the rrLU on a rank-deficient (CP-rank-K) Pi matrix: the same matrix factorised
several times with the shadow search on and once with it off must give bitwise the same result.

  python scripts/determinism_check.py [m] [K] [reps]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tensorcrossinterpolation.jl_amd"))

import numpy as np  # noqa: E402

import tci_amd as T  # noqa: E402

m = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
K = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
L, d = 12, 32
rng = np.random.default_rng(2)
f = T.cp_function(0.5 + rng.random((K, L, d)))
I = rng.integers(1, d + 1, size=(m, 6)).astype(np.int32)
J = rng.integers(1, d + 1, size=(m, 6)).astype(np.int32)
Pi, mx = f.pi(I, J, 0)
print("Pi", Pi.shape, "max", mx, flush=True)
ctx = T.context()
res = []
for r in range(reps + 1):
    shadow = r < reps
    ctx.check(ctx.lib.tci_set_rrlu_shadow(ctx.h, int(shadow)))
    lu = T.rrlu(Pi, maxrank=K + 8, ctx=ctx)
    res.append(lu)
    print(f"run {r} shadow={shadow} npivot={lu.npivot} error={lu.error!r} "
          f"last pivots={T.pivoterrors(lu)[-4:]}", flush=True)
ref = res[-1]
for r, lu in enumerate(res[:-1]):
    same = (lu.npivot == ref.npivot and np.array_equal(lu.rowpermutation, ref.rowpermutation)
            and np.array_equal(lu.colpermutation, ref.colpermutation) and np.array_equal(lu.L, ref.L)
            and np.array_equal(lu.U, ref.U))
    k = next((i for i in range(min(lu.npivot, ref.npivot))
              if lu.rowpermutation[i] != ref.rowpermutation[i] or lu.colpermutation[i] != ref.colpermutation[i]),
             None)
    print(f"run {r} vs exact: bitwise {'SAME' if same else 'DIFFERENT'}; first differing pivot {k}")
