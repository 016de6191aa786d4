"""The native sweep driver (tci_tci2_sweep2site, tci_sweep.cpp) against sweep2site's host loop
(tensorci2.py) and the oracle: identical ranks, pivot sets, errors and maxsamplevalue, for the
default flow (back-and-forth, non-strictly nested: unions with the previous sweep's sets), the
forward and strictly nested variants, and a run with global pivots (history + extra pivots).
Reference: tensorci2.jl:1195-1258 (sweep2site!), :825-930 (updatepivots!)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

T = pytest.importorskip("tci_amd")
import tci_amd.tensorci2 as TT  # noqa: E402


def _run(f, ld, native, **kw):
    TT.NATIVE_SWEEP = native
    try:
        return T.crossinterpolate2(f, ld, [T.optfirstpivot(f, ld)], **kw)
    finally:
        TT.NATIVE_SWEEP = True


CASES = [
    ("lorentz8", lambda ctx: T.lorentz([10] * 8, ctx=ctx), [10] * 8, dict(tolerance=1e-8, nsearchglobalpivot=0)),
    ("qosc24", lambda ctx: T.quantics_osc(24, ctx=ctx), [2] * 24, dict(tolerance=1e-8, nsearchglobalpivot=0)),
    ("lorentz_forward", lambda ctx: T.lorentz([6] * 6, ctx=ctx), [6] * 6,
     dict(tolerance=1e-10, nsearchglobalpivot=0, sweepstrategy="forward")),
    ("lorentz_strict", lambda ctx: T.lorentz([6] * 6, ctx=ctx), [6] * 6,
     dict(tolerance=1e-10, nsearchglobalpivot=0, strictlynested=True)),
    ("lorentz_maxbond", lambda ctx: T.lorentz([10] * 6, ctx=ctx), [10] * 6,
     dict(tolerance=1e-14, maxbonddim=7, maxiter=5, nsearchglobalpivot=0)),
    ("lorentz_global", lambda ctx: T.lorentz([8] * 6, ctx=ctx), [8] * 6, dict(tolerance=1e-10, nsearchglobalpivot=5)),
]


@pytest.mark.parametrize("name", [c[0] for c in CASES])
def test_native_equals_host_loop(name):
    ctx = T.context(0)
    _, mk, ld, kw = next(c for c in CASES if c[0] == name)
    f = mk(ctx)
    extra = {"rng": np.random.default_rng(4)} if kw.get("nsearchglobalpivot") else {}
    t1, r1, e1 = _run(f, ld, True, **kw, **extra)
    extra = {"rng": np.random.default_rng(4)} if kw.get("nsearchglobalpivot") else {}
    t2, r2, e2 = _run(f, ld, False, **kw, **extra)
    assert r1 == r2 and list(e1) == list(e2)
    assert t1.maxsamplevalue == t2.maxsamplevalue
    for b in range(len(ld)):
        assert np.array_equal(t1.Iset[b], t2.Iset[b]) and np.array_equal(t1.Jset[b], t2.Jset[b])
        assert np.array_equal(t1.sitetensors[b], t2.sitetensors[b])
