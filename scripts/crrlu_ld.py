"""ComplexF64 rrLU on device matrices with different leading dimensions (power-of-two column
strides vs padded): python scripts/crrlu_ld.py [m n r]..."""
import ctypes as C
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tensorcrossinterpolation.jl_amd"))
import tci_amd as T  # noqa: E402

ctx = T.Context(0)
for m, n, r in ((4096, 4096, 256), (8192, 8192, 256)):
    for pad in (0, 16, 64):
        ld = m + pad
        A = T.DeviceMatrix(2 * m, n, ctx=ctx, ld=2 * ld)
        A.fill_uniform(seed=0)
        W = T.DeviceMatrix(2 * m, n, ctx=ctx, ld=2 * ld)
        npv, err = C.c_int64(), C.c_double()
        ts = []
        for _ in range(3):
            W.copy_from(A)
            ctx.synchronize()
            t0 = time.perf_counter()
            ctx.check(ctx.lib.tci_rrlu_c128_inplace_d(ctx.h, W.ptr, m, n, ld, r, 1e-14, 0.0, 1, None, None,
                                                      C.byref(npv), C.byref(err), None))
            ts.append(time.perf_counter() - t0)
        print(f"{m}x{n} r={npv.value} ld={ld}: {min(ts) * 1e3:.1f} ms", flush=True)
        A.free()
        W.free()
