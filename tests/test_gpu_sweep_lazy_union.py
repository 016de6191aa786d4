"""The small sweep's lazy union (tci_sweep_small.hip, legs with d >= 4: the kronecker products are
never materialised; rows, states and new sets are read by descriptor) gives bitwise the same
TCI2 as the materialised union (TCI_SW_LAZYU=0 on a second context): sets, histories, errors,
ranks, maxsample and site tensors, over kinds with d = 2 (materialised either way), 4, 10 and 16,
with and without strict nesting (the extras are what the lazy union dedups)."""
import os

import numpy as np
import pytest

T = pytest.importorskip("tci_amd")
from tci_amd import _lib  # noqa: E402

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctxs():
    lazy = _lib.context()
    old = os.environ.get("TCI_SW_LAZYU")
    os.environ["TCI_SW_LAZYU"] = "0"
    try:
        eager = _lib.Context(int(os.environ.get("TCI_DEVICE", "0")))
    finally:
        if old is None:
            del os.environ["TCI_SW_LAZYU"]
        else:
            os.environ["TCI_SW_LAZYU"] = old
    yield lazy, eager
    eager.close()


CASES = [
    ("lorentz d=10", lambda ctx: T.lorentz([10] * 8, ctx=ctx), [10] * 8, None, dict(tolerance=1e-8)),
    ("gauss d=16", lambda ctx: T.gauss([16] * 12, 0.05, 8.5, ctx=ctx), [16] * 12, [[8] * 12],
     dict(tolerance=1e-10, maxbonddim=64)),
    ("lorentz d=4", lambda ctx: T.lorentz([4] * 14, ctx=ctx), [4] * 14, None, dict(tolerance=1e-10)),
    ("qosc d=2", lambda ctx: T.quantics_osc(20, ctx=ctx), [2] * 20, None, dict(tolerance=1e-8)),
]


@pytest.mark.parametrize("name,make,ld,p0,kw", CASES, ids=[c[0] for c in CASES])
@pytest.mark.parametrize("strict", [False, True])
def test_lazy_union_bitwise(ctxs, name, make, ld, p0, kw, strict):
    outs = []
    for ctx in ctxs:
        f = make(ctx)
        piv = p0 if p0 is not None else [T.optfirstpivot(f, ld)]
        tci, ranks, errors = T.crossinterpolate2(f, ld, piv, nsearchglobalpivot=0, strictlynested=strict, **kw)
        outs.append((tci, ranks, errors))
    (a, ra, ea), (b, rb, eb) = outs
    assert ra == rb
    assert np.array_equal(np.asarray(ea), np.asarray(eb))
    assert a.maxsamplevalue == b.maxsamplevalue
    for p in range(len(ld)):
        assert np.array_equal(a.Iset[p], b.Iset[p]) and np.array_equal(a.Jset[p], b.Jset[p])
        assert np.array_equal(np.asarray(a.sitetensors[p]).view(np.uint64), np.asarray(b.sitetensors[p]).view(np.uint64))
    if a.Iset_history:
        for p in range(len(ld)):
            assert np.array_equal(a.Iset_history[-1][p], b.Iset_history[-1][p])
            assert np.array_equal(a.Jset_history[-1][p], b.Jset_history[-1][p])
