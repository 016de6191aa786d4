"""optimize! as one chain of device launches (tci_tci2_optimize_small: the iterations' state handed
over in device memory, abstol / pivoterror / rank / convergencecriterion on the device, then the
closing sweep1site!) against the per-iteration path (TensorCI2's Python loop over native
sweep2site! calls, tensorci2.OPTIMIZE_CHAIN = False): bitwise the same ranks, errors, index sets,
histories, maxsample, pivot / bond errors and site tensors -- with solved and lazy fills, strict
nesting, a maxbonddim cap, maxiter reached without convergence, normalizeerror off, and a chain that
stops early because a bond outgrows the small path (the loop then continues on the host)."""
import numpy as np
import pytest

T = pytest.importorskip("tci_amd")
from tci_amd import tensorci2 as T2  # noqa: E402

pytestmark = pytest.mark.gpu


def _run(chain, make, ld, p0, kw):
    old = T2.OPTIMIZE_CHAIN
    T2.OPTIMIZE_CHAIN = chain
    try:
        f = make()
        piv = p0 if p0 is not None else [T.optfirstpivot(f, ld)]
        return T.crossinterpolate2(f, ld, piv, nsearchglobalpivot=0, **kw)
    finally:
        T2.OPTIMIZE_CHAIN = old


def _same(a, b, ld):
    (ta, ra, ea), (tb, rb, eb) = a, b
    assert ra == rb
    assert np.array_equal(np.asarray(ea, float).view(np.uint64), np.asarray(eb, float).view(np.uint64))
    assert ta.maxsamplevalue == tb.maxsamplevalue
    assert np.array_equal(np.asarray(ta.pivoterrors), np.asarray(tb.pivoterrors))
    assert np.array_equal(np.asarray(ta.bonderrors), np.asarray(tb.bonderrors))
    for p in range(len(ld)):
        assert np.array_equal(ta.Iset[p], tb.Iset[p]) and np.array_equal(ta.Jset[p], tb.Jset[p])
        assert np.array_equal(np.asarray(ta.sitetensors[p]).view(np.uint64),
                              np.asarray(tb.sitetensors[p]).view(np.uint64))
    assert len(ta.Iset_history) == len(tb.Iset_history)
    if ta.Iset_history:
        for p in range(len(ld)):
            assert np.array_equal(ta.Iset_history[-1][p], tb.Iset_history[-1][p])
            assert np.array_equal(ta.Jset_history[-1][p], tb.Jset_history[-1][p])


CASES = [
    ("C1 lorentz", lambda: T.lorentz([10] * 8), [10] * 8, None, dict(tolerance=1e-8)),
    ("C3 gauss", lambda: T.gauss([16] * 20, 0.05, 8.5), [16] * 20, [[8] * 20], dict(tolerance=1e-10, maxbonddim=512)),
    ("C4 qosc", lambda: T.quantics_osc(40), [2] * 40, None, dict(tolerance=1e-8)),
    ("lazy fill", lambda: T.lorentz([10] * 8), [10] * 8, None, dict(tolerance=1e-8, lazy_sitetensors=True)),
    ("strict", lambda: T.quantics_osc(24), [2] * 24, None, dict(tolerance=1e-8, strictlynested=True)),
    ("maxbonddim cap", lambda: T.quantics_osc(24), [2] * 24, None, dict(tolerance=1e-12, maxbonddim=6)),
    ("maxiter", lambda: T.quantics_osc(30), [2] * 30, None, dict(tolerance=1e-14, maxiter=4)),
    ("no normalize", lambda: T.lorentz([6] * 10, coeff=3.0), [6] * 10, None,
     dict(tolerance=1e-9, normalizeerror=False)),
    ("ncheck 1", lambda: T.lorentz([10] * 8), [10] * 8, None, dict(tolerance=1e-8, ncheckhistory=1)),
]


@pytest.mark.parametrize("name,make,ld,p0,kw", CASES, ids=[c[0] for c in CASES])
def test_chain_equals_per_iteration(name, make, ld, p0, kw):
    _same(_run(True, make, ld, p0, kw), _run(False, make, ld, p0, kw), ld)


def test_chain_stops_where_a_bond_outgrows_the_small_path():
    # ranks grow past the one-workgroup rrLU within a few iterations: the chain hands the state back
    # and the loop finishes on the host -- same results as without the chain
    mk = lambda: T.lorentz([16] * 6)  # noqa: E731
    ld = [16] * 6
    kw = dict(tolerance=1e-13)
    _same(_run(True, mk, ld, None, kw), _run(False, mk, ld, None, kw), ld)


def test_chain_used_on_c4():
    """the chain actually runs (not a silent fallback): one native call covers the whole loop"""
    f = T.quantics_osc(40)
    ld = [2] * 40
    tci = T2.TensorCI2.from_function(f, ld, [T.optfirstpivot(f, ld)])
    r = tci._optimize_native(f, 1e-8, T2.INT64_MAX, 20, 3, True, False, False)
    assert r is not None
    nd, errs, rks, ended, s1done, errnorm = r
    assert ended and s1done and nd >= 3 and len(errs) == nd and len(rks) == nd
