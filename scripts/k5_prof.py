"""K5 (setsitetensor!'s solve, T = Pi1 P^-1) at the C5 shape, for a kernel trace:
   rocprofv3 --kernel-trace --stats -- python3 scripts/k5_prof.py [r R reps]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tensorcrossinterpolation.jl_amd"))
import tci_amd as T  # noqa: E402
from tci_amd import _lib  # noqa: E402

r, R, reps = (int(x) for x in (sys.argv[1:] + ["1024", "32768", "3"][len(sys.argv[1:]):]))
ctx = _lib.context()
P0 = T.DeviceMatrix(r, r, ctx=ctx, ld=r)
P0.fill_uniform(seed=6)
P = T.DeviceMatrix(r, r, ctx=ctx, ld=r)
Pi1 = T.DeviceMatrix(R, r, ctx=ctx, ld=R)
Pi1.fill_uniform(seed=7)
Tm = T.DeviceMatrix(R, r, ctx=ctx, ld=R)
P.copy_from(P0)
T.sitetensor_solve_device(P, Pi1, Tm)
ctx.set_timing(True)
t0 = time.perf_counter()
for _ in range(reps):
    P.copy_from(P0)
    T.sitetensor_solve_device(P, Pi1, Tm)
wall = time.perf_counter() - t0
kms, kn = ctx.kernel_stats(20)
ctx.set_timing(False)
print(f"r {r} R {R}: {kms / kn:.3f} ms per solve (HIP events), wall {wall / reps * 1e3:.3f} ms")
