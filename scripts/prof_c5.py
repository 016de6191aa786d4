"""Host-side split of config 5 as stated (12d CP-rank-1024, d = 32, maxbonddim 1024, maxiter 3, the
reference's fill): wall time per ABI entry (a timing proxy on ctx.lib) and the Python functions by
cumulative time.   python scripts/prof_c5.py [lazy]"""
import cProfile
import io
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tensorcrossinterpolation.jl_amd"))
sys.path.insert(0, os.path.join(ROOT, "scripts"))
import numpy as np  # noqa: E402

import tci_amd as T  # noqa: E402
from tci_amd import _lib as L  # noqa: E402
from prof_small_py import _TimedLib  # noqa: E402

lazy = "lazy" in sys.argv[1:]
rng = np.random.default_rng(2)
K, Ls, d = 1024, 12, 32
f = T.cp_function(0.5 + rng.random((K, Ls, d)))
p0 = T.optfirstpivot(f, [d] * Ls)
kw = dict(tolerance=1e-10, maxbonddim=1024, maxiter=3, nsearchglobalpivot=0, lazy_sitetensors=lazy)
ctx = L.context()
timed = _TimedLib(ctx.lib)
ctx.lib = timed
pr = cProfile.Profile()
t0 = time.perf_counter()
pr.enable()
T.crossinterpolate2(f, [d] * Ls, [p0], **kw)
pr.disable()
wall = time.perf_counter() - t0
ctx.lib = timed._lib
abi = sum(v[1] for v in timed.acc.values())
print(f"C5 ({'lazy' if lazy else 'reference work'}): wall {wall:.3f} s, ABI {abi:.3f} s, Python {wall - abi:.3f} s")
for k, (n, t) in sorted(timed.acc.items(), key=lambda kv: -kv[1][1])[:16]:
    print(f"   {k:40s} {n:5d} calls {t:9.3f} s")
s = io.StringIO()
pstats.Stats(pr, stream=s).sort_stats("cumulative").print_stats(30)
print(s.getvalue())
