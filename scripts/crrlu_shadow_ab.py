"""ComplexF64 rrLU on device matrices with the certified shadow search on and off:
time per factorisation and equality of the pivots / pivot errors between the two settings at the
benchmarked sizes. python scripts/crrlu_shadow_ab.py [m,n,r ...]"""
import ctypes as C
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tensorcrossinterpolation.jl_amd"))
import tci_amd as T  # noqa: E402

ctx = T.Context(0)
sizes = [tuple(int(v) for v in a.split(",")) for a in sys.argv[1:]] or [(4096, 4096, 256), (8192, 8192, 256)]
for m, n, r in sizes:
    A = T.DeviceMatrix(2 * m, n, ctx=ctx)
    A.fill_uniform(seed=0)
    W = T.DeviceMatrix(2 * m, n, ctx=ctx)
    res = {}
    for sh in (1, 0):
        ctx.check(ctx.lib.tci_set_c128_shadow(ctx.h, sh))
        npv, err = C.c_int64(), C.c_double()
        rp, cp, pe = np.zeros(m, np.int64), np.zeros(n, np.int64), np.zeros(r + 1)
        ts = []
        for _ in range(3):
            W.copy_from(A)
            ctx.synchronize()
            t0 = time.perf_counter()
            ctx.check(ctx.lib.tci_rrlu_c128_inplace_d(ctx.h, W.ptr, m, n, W.ld // 2, r, 1e-14, 0.0, 1,
                                                      T._lib.ptr(rp), T._lib.ptr(cp), C.byref(npv),
                                                      C.byref(err), T._lib.ptr(pe)))
            ts.append(time.perf_counter() - t0)
        res[sh] = (npv.value, rp.copy(), cp.copy(), pe.copy(), err.value)
        print(f"{m}x{n} r={npv.value} shadow={sh}: {min(ts) * 1e3:.2f} ms", flush=True)
    a, b = res[1], res[0]
    same = (a[0] == b[0] and np.array_equal(a[1], b[1]) and np.array_equal(a[2], b[2])
            and np.array_equal(a[3], b[3]) and a[4] == b[4])
    print(f"{m}x{n}: shadow on == off (pivots, pivot errors, error): {same}", flush=True)
    A.free()
    W.free()
    if not same:
        sys.exit(1)
ctx.check(ctx.lib.tci_set_c128_shadow(ctx.h, 1))
