"""Diagnostic: the first pivot at which the persistent epoch launch's rrLU differs from the per-pass
launches' (and the oracle's) on one matrix. python scripts/persist_debug.py [m n r nb epochs]"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tensorcrossinterpolation.jl_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
import numpy as np  # noqa: E402

import oracle_lib as O  # noqa: E402
import tci_amd as T  # noqa: E402

m, n, r, nb, ep = (int(x) for x in (sys.argv[1:6] if len(sys.argv) > 5 else (2100, 1900, 150, 10, 3)))
A = O.fill_uniform(m * n, seed=7 + nb + 10 * ep).reshape((m, n), order="F")
ref = O.OracleLU(A, maxrank=r)
for persist in (0, 1):
    c = T.Context(0)
    c.check(c.lib.tci_set_rrlu_small(c.h, 0))
    c.check(c.lib.tci_set_rrlu_mid(c.h, 0))
    c.check(c.lib.tci_set_rrlu_persist(c.h, persist))
    c.check(c.lib.tci_set_rrlu_flush(c.h, nb))
    c.check(c.lib.tci_set_rrlu_epochs(c.h, ep))
    lu = T.rrlu(A, ctx=c, maxrank=r)
    rp, cp = lu.rowpermutation - 1, lu.colpermutation - 1
    bad = [k for k in range(min(lu.npivot, ref.npivot)) if rp[k] != ref.rowpermutation[k] or cp[k] != ref.colpermutation[k]]
    Ld = np.nonzero(np.any(lu.L != ref.L, axis=0))[0] if lu.L.shape == ref.L.shape else "shape"
    Ud = np.nonzero(np.any(lu.U != ref.U, axis=1))[0] if lu.U.shape == ref.U.shape else "shape"
    print(f"persist={persist} kinds={os.environ.get('TCI_EPOCH_KINDS', '3')} npivot {lu.npivot}/{ref.npivot} "
          f"first bad pivot {bad[:5]} L cols differ {list(Ld)[:8]} U rows differ {list(Ud)[:8]} "
          f"faulted={c.lib.tci_rrlu_persist_faulted(c.h)}")
    print("   rows", list(rp[:8]), "cols", list(cp[:8]), "piv", [float(x) for x in np.diag(lu.U)[:5]] if hasattr(lu, 'U') else '')
    print("   ref  ", list(ref.rowpermutation[:8]), "cols", list(ref.colpermutation[:8]))
    c.close()
