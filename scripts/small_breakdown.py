"""Where the wall time of the small TCI2 configs (C3 gauss20d, C4 qosc40) goes on the GPU path:
sweep2site (native per-bond loop), fillsitetensors, the final sweep1site, the rest (Python).

  python scripts/small_breakdown.py
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


def wrap(cls, name):
    fn = getattr(cls, name)

    def w(*a, **k):
        t0 = time.perf_counter()
        try:
            return fn(*a, **k)
        finally:
            acc[name] += time.perf_counter() - t0
            cnt[name] += 1
    setattr(cls, name, w)


for nm in ("_sweep2site_native", "fillsitetensors", "sweep1site", "sweep2site"):
    wrap(TT.TensorCI2, nm)


def case(name, f, ld, p0, **kw):
    T.crossinterpolate2(f, ld, [p0], **dict(kw, maxiter=1))
    acc.clear()
    cnt.clear()
    t0 = time.perf_counter()
    tci, ranks, errors = T.crossinterpolate2(f, ld, [p0], **kw)
    wall = time.perf_counter() - t0
    print(json.dumps({"config": name, "wall_ms": round(wall * 1e3, 3), "ranks": ranks,
                      "parts_ms": {k: round(v * 1e3, 3) for k, v in acc.items()}, "calls": dict(cnt)}))


fq = T.quantics_osc(40)
case("C4_qosc40", fq, [2] * 40, T.optfirstpivot(fq, [2] * 40), tolerance=1e-8, nsearchglobalpivot=0)
case("C3_gauss20d", T.gauss([16] * 20, 0.05, 8.5), [16] * 20, [8] * 20, tolerance=1e-10, maxbonddim=512,
     nsearchglobalpivot=0)
