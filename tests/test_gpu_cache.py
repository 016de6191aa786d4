"""CachedFunction's memo on the device (tci_cache_*, tci_cache.hip; cachedfunction.jl:53-302), through
the C ABI: a Pi block served through the memo equals the direct batch evaluation bit for bit (same
device integrand, same values), the batch's distinct misses are evaluated once (repeats within a
batch included), a second pass is all hits, growth (rehash) keeps every entry, clearcache! empties
it, and a TCI2 run through the memo reproduces the run without it (test_cachedfunction.jl's own
checks, :50-90, on the device)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

T = pytest.importorskip("tci_amd")


@pytest.fixture(scope="module")
def ctx():
    c = T.Context(0)
    yield c
    c.close()


@pytest.mark.parametrize("kind", ["lorentz", "qosc", "tt"])
@pytest.mark.parametrize("M", [0, 1])
def test_memo_pi_bitwise_and_counts(ctx, kind, M):
    rng = np.random.default_rng(3 + M)
    if kind == "lorentz":
        ld = [6] * 7
        f = T.lorentz(ld, ctx=ctx)
    elif kind == "qosc":
        ld = [2] * 16
        f = T.quantics_osc(16, ctx=ctx)
    else:
        ld = [3] * 6
        cores = [rng.standard_normal((1 if t == 0 else 4, 3, 1 if t == 5 else 4)) for t in range(6)]
        f = T.tensortrain_function(cores, ctx=ctx)
    L = len(ld)
    nl = 3
    nr = L - nl - M
    I = np.stack([rng.integers(1, ld[t] + 1, 40) for t in range(nl)], 1).astype(np.int32)
    J = np.stack([rng.integers(1, ld[nl + M + t] + 1, 30) for t in range(nr)], 1).astype(np.int32)
    I[5] = I[0]  # repeated rows: the same keys twice in one batch
    J[7] = J[2]
    ref, rmx = f.pi(I, J, M)
    cf = T.CachedFunction(f, ld)
    assert cf._memo is not None
    got, mx = cf.pi(I, J, M)
    assert np.array_equal(got, ref) and mx == rmx
    D = ld[nl] if M else 1
    distinct = len({(tuple(I[i]), c, tuple(J[j])) for i in range(len(I)) for c in range(D) for j in range(len(J))})
    assert cf.nmiss_last == distinct and cf.ncacheddata() == distinct
    got2, mx2 = cf.pi(I, J, M)
    assert cf.nmiss_last == 0 and np.array_equal(got2, ref) and mx2 == rmx
    # cacheddata: the stored values are f's at the decoded index sets
    data = cf.cacheddata()
    keys = list(data)[:20]
    vals = f.points(np.asarray(keys, np.int32))
    assert np.array_equal(np.array([data[k] for k in keys]), vals)
    cf.clearcache()
    assert cf.ncacheddata() == 0
    got3, _ = cf.pi(I, J, M)
    assert cf.nmiss_last == distinct and np.array_equal(got3, ref)


def test_memo_growth_keeps_entries(ctx):
    ld = [4] * 10
    f = T.lorentz(ld, ctx=ctx)
    cf = T.CachedFunction(f, ld)
    rng = np.random.default_rng(9)
    seen = set()
    for _ in range(6):  # 6 x 4096 points: the table starts at 8192 slots and must grow
        X = rng.integers(1, 5, (4096, 10)).astype(np.int32)
        v = cf.points(X)
        assert np.array_equal(v, f.points(X))
        seen |= {tuple(x) for x in X}
    assert cf.ncacheddata() == len(seen)
    X = np.array(sorted(seen)[:500], np.int32)
    cf.points(X)
    assert cf.nmiss_last == 0


def test_memo_tci2_matches_uncached(ctx):
    ld = [10] * 5
    f = T.lorentz(ld, ctx=ctx)
    cf = T.CachedFunction(f, ld)
    kw = dict(tolerance=1e-10, maxiter=20, nsearchglobalpivot=0)
    t1, r1, e1 = T.crossinterpolate2(f, ld, [[1] * 5], **kw)
    t2, r2, e2 = T.crossinterpolate2(cf, ld, [[1] * 5], **kw)
    assert r1 == r2 and list(e1) == list(e2)
    for b in range(5):
        assert np.array_equal(t1.Iset[b], t2.Iset[b]) and np.array_equal(t1.Jset[b], t2.Jset[b])
    n = cf.ncacheddata()
    T.crossinterpolate2(cf, ld, [[1] * 5], **kw)
    assert cf.ncacheddata() == n  # the second run is served from the memo
