"""Host-side profile of the small TCI2 configs (C3 gauss20d, C4 qosc40): cProfile of one
crossinterpolate2 after a warm-up, the top functions by own time, and a per-phase wall split
(the native sweep's ABI call vs the Python around it).

  python scripts/prof_small_py.py [C3|C4]
"""
import cProfile
import io
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tensorcrossinterpolation.jl_amd"))

import tci_amd as T  # noqa: E402

class _TimedLib:
    """ctx.lib proxy: wall time and calls per ABI entry"""

    def __init__(self, lib):
        self._lib, self.acc = lib, {}

    def __getattr__(self, name):
        fn = getattr(self._lib, name)
        if not callable(fn):
            return fn

        def call(*a, _fn=fn, _n=name):
            t = time.perf_counter()
            try:
                return _fn(*a)
            finally:
                c = self.acc.setdefault(_n, [0, 0.0])
                c[0] += 1
                c[1] += time.perf_counter() - t
        return call


def main():
    which = sys.argv[1:] or ["C3", "C4"]
    cases = {}
    if "C4" in which:
        fq = T.quantics_osc(40)
        cases["C4"] = (fq, [2] * 40, [T.optfirstpivot(fq, [2] * 40)], dict(tolerance=1e-8, nsearchglobalpivot=0))
    if "C3" in which:
        cases["C3"] = (T.gauss([16] * 20, 0.05, 8.5), [16] * 20, [[8] * 20],
                       dict(tolerance=1e-10, maxbonddim=512, nsearchglobalpivot=0))


    from tci_amd import _lib as L  # noqa: E402
    ctx = L.context()
    timed = _TimedLib(ctx.lib)
    for name, (f, ld, p0, kw) in cases.items():
        for _ in range(3):
            T.crossinterpolate2(f, ld, p0, **kw)
        t0 = time.perf_counter()
        T.crossinterpolate2(f, ld, p0, **kw)
        wall = time.perf_counter() - t0
        ctx.lib = timed
        timed.acc.clear()
        t0 = time.perf_counter()
        T.crossinterpolate2(f, ld, p0, **kw)
        wt = time.perf_counter() - t0
        ctx.lib = timed._lib
        abi = sum(v[1] for v in timed.acc.values())
        print(f"== {name}: ABI split (one run, {wt * 1e3:.3f} ms with the proxy): ABI {abi * 1e3:.3f} ms, "
              f"Python {(wt - abi) * 1e3:.3f} ms")
        for k, (n, t) in sorted(timed.acc.items(), key=lambda kv: -kv[1][1])[:14]:
            print(f"   {k:40s} {n:4d} calls {t * 1e3:8.3f} ms")
        pr = cProfile.Profile()
        pr.enable()
        T.crossinterpolate2(f, ld, p0, **kw)
        pr.disable()
        s = io.StringIO()
        pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(25)
        print(f"== {name}: wall {wall * 1e3:.3f} ms (unprofiled)")
        print(s.getvalue())


if __name__ == "__main__":
    main()
