"""The quantics-oscillatory Pi assembly of bench.py's extras alone (8192 x 8192, 40 legs), for
rocprofv3 PMC passes (fp64 VALU instruction counts -> flops per element, bench.py qosc_roofline):
python scripts/qosc_assembly.py [reps]"""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tensorcrossinterpolation.jl_amd"))
import numpy as np  # noqa: E402

import tci_amd as T  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
ctx = T.Context(0)
m = n = 8192
rng = np.random.default_rng(1)
rng.integers(1, 11, (m, 10)), rng.integers(1, 11, (n, 10))  # bench.py's draws before these
Ib = rng.integers(1, 3, (m, 20)).astype(np.int32)
Jb = rng.integers(1, 3, (n, 20)).astype(np.int32)
f = T.GPUBatchEvaluator(5, T.batcheval.QOSC_PARAMS, [2] * 40, ctx=ctx)
dm = T.DeviceMatrix(m, n, ctx=ctx)
mx = C.c_double()
for _ in range(reps):
    ctx.check(ctx.lib.tci_batcheval_d(ctx.h, f.h, T._lib.ptr(Ib), m, 20, T._lib.ptr(Jb), n, 20, 0, dm.ptr, dm.ld,
                                      C.byref(mx)))
ctx.synchronize()
print("elements per launch", m * n, "launches", reps, flush=True)
