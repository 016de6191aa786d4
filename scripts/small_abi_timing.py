"""Host-side timeline of the small TCI2 configs: wall time of every libtci_hip ABI call made while
crossinterpolate2 runs C4 (quantics 40 legs) and C3 (separable Gaussian 20 legs), grouped by
entry point, next to the Python-level parts (sweep2site / sweep1site). Run it under
`rocprofv3 --kernel-trace --stats` for the kernel side.

  python scripts/small_abi_timing.py
"""
import json
import os
import sys
import time
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tensorcrossinterpolation.jl_amd"))

import tci_amd as T  # noqa: E402
from tci_amd import tensorci2 as TT  # noqa: E402

acc = defaultdict(float)
cnt = defaultdict(int)


def wrap_lib(lib):
    for nm in dir(lib):
        if not nm.startswith("tci_"):
            continue
        fn = getattr(lib, nm)

        def w(*a, _fn=fn, _nm=nm):
            t0 = time.perf_counter()
            try:
                return _fn(*a)
            finally:
                acc["abi:" + _nm] += time.perf_counter() - t0
                cnt["abi:" + _nm] += 1
        try:
            setattr(lib, nm, w)
        except Exception:
            pass


def wrap(cls, name):
    fn = getattr(cls, name)

    def w(*a, **k):
        t0 = time.perf_counter()
        try:
            return fn(*a, **k)
        finally:
            acc["py:" + name] += time.perf_counter() - t0
            cnt["py:" + name] += 1
    setattr(cls, name, w)


for nm in ("_sweep2site_native", "sweep1site", "sweep2site", "fillsitetensors", "optimize"):
    wrap(TT.TensorCI2, nm)


def case(name, f, ld, p0, **kw):
    T.crossinterpolate2(f, ld, [p0], **kw)  # warm-up: same sizes, every buffer allocated
    acc.clear()
    cnt.clear()
    t0 = time.perf_counter()
    _, ranks, _ = T.crossinterpolate2(f, ld, [p0], **kw)
    wall = time.perf_counter() - t0
    parts = {k: [round(v * 1e3, 3), cnt[k]] for k, v in sorted(acc.items(), key=lambda kv: -kv[1])}
    print(json.dumps({"config": name, "wall_ms": round(wall * 1e3, 3), "ranks": ranks, "ms_calls": parts}))


fq = T.quantics_osc(40)
wrap_lib(fq.ctx.lib)
case("C4_qosc40", fq, [2] * 40, T.optfirstpivot(fq, [2] * 40), tolerance=1e-8, nsearchglobalpivot=0)
case("C3_gauss20d", T.gauss([16] * 20, 0.05, 8.5), [16] * 20, [8] * 20, tolerance=1e-10, maxbonddim=512,
     nsearchglobalpivot=0)
