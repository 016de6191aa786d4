"""rrLU repeatability over shapes (pass pipeline): each shape factorised 3 times (shadow on) and
once with the shadow off; prints whether all agree bitwise."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tensorcrossinterpolation.jl_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import numpy as np  # noqa: E402

import tci_amd as T  # noqa: E402

ctx = T.context()
ctx.check(ctx.lib.tci_set_rrlu_small(ctx.h, 0))
ctx.check(ctx.lib.tci_set_rrlu_mid(ctx.h, 0))
shapes = [tuple(int(x) for x in s.split("x")) for s in sys.argv[1:]] or [
    (8192, 8192, 256), (8216, 8192, 256), (8192, 8216, 256), (8704, 8192, 256), (4096, 8704, 128), (2000, 9000, 64)]
rng = np.random.default_rng(0)
for (m, n, r) in shapes:
    A = np.asfortranarray(rng.random((m, n)))
    outs = []
    for rep in range(4):
        ctx.check(ctx.lib.tci_set_rrlu_shadow(ctx.h, int(rep < 3)))
        lu = T.rrlu(A, maxrank=r, ctx=ctx)
        outs.append((T.rowindices(lu).copy(), T.colindices(lu).copy(), lu.L.copy(), lu.U.copy()))
    agree = [all(np.array_equal(a, b) for a, b in zip(outs[i], outs[3])) for i in range(3)]
    first = []
    for i in range(3):
        d = np.nonzero((outs[i][0] != outs[3][0]) | (outs[i][1] != outs[3][1]))[0]
        first.append(int(d[0]) if len(d) else None)
    print(f"{m}x{n} r={r}: shadow runs agree with exact: {agree}; first differing pivot {first}", flush=True)
