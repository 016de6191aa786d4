"""Cross-check of the fused 2-site update (tci_update_pivots_h) inside a TCI2 sweep: every call is
repeated as Pi = f.pi(rows, cols) + a standalone rrlu on that Pi, and the pivots compared."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tensorcrossinterpolation.jl_amd"))

import numpy as np  # noqa: E402

import tci_amd as T  # noqa: E402
import tci_amd.tensorci2 as TT  # noqa: E402

orig = TT.update_pivots_device
calls = [0]


def checked(f, rows, cols, maxrank, reltol, abstol, leftorth, want_factors, want_left=True, want_right=True):
    res = orig(f, rows, cols, maxrank, reltol, abstol, leftorth, want_factors, want_left, want_right)
    calls[0] += 1
    Pi, mx = f.pi(np.asarray(rows, np.int32), np.asarray(cols, np.int32), 0)
    lu = T.rrlu(np.asfortranarray(Pi), maxrank=int(min(maxrank, 2**62)), reltol=reltol, abstol=abstol,
                leftorthogonal=leftorth)
    lu2 = T.rrlu(np.asfortranarray(Pi), maxrank=int(min(maxrank, 2**62)), reltol=reltol, abstol=abstol,
                 leftorthogonal=leftorth)
    ri = T.rowindices(lu) - 1
    ci = T.colindices(lu) - 1
    same12 = np.array_equal(T.rowindices(lu), T.rowindices(lu2)) and np.array_equal(T.colindices(lu), T.colindices(lu2))
    ok = (res["npivot"] == lu.npivot and np.array_equal(np.asarray(res["rowidx"]) - 0, ri + 1)
          and np.array_equal(np.asarray(res["colidx"]), ci + 1)) or (
        res["npivot"] == lu.npivot and np.array_equal(np.asarray(res["rowidx"]), ri)
        and np.array_equal(np.asarray(res["colidx"]), ci))
    if not ok or not same12 or mx != res["maxabs"]:
        print(f"call {calls[0]}: Pi {Pi.shape} maxrank {maxrank} leftorth {leftorth}: fused np={res['npivot']} "
              f"standalone np={lu.npivot}; pivots equal {ok}; standalone repeat equal {same12}; "
              f"max {res['maxabs']} vs {mx}; fused rows[:5] {np.asarray(res['rowidx'])[:5]} standalone {ri[:5]}",
              flush=True)
    return res


TT.update_pivots_device = checked
K = int(sys.argv[1]) if len(sys.argv) > 1 else 256
rng = np.random.default_rng(2)
L, d = 12, 32
f = T.cp_function(0.5 + rng.random((K, L, d)))
p0 = T.optfirstpivot(f, [d] * L)
for r in range(2):
    tci, ranks, errors = T.crossinterpolate2(f, [d] * L, [p0], tolerance=1e-10, maxbonddim=K, maxiter=3,
                                             nsearchglobalpivot=0)
    print("run", r, ranks, errors, "calls", calls[0], flush=True)
