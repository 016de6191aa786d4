"""GPU parity of the ComplexF64 rrLU (tci_rrlu_c128_h, tci_rrlu_c128.hip) with the CPU oracle
(orc_rrlu_c128): bit-exact permutations, L, U, npivot, lu.error and pivot errors -- the device
restates Julia's complex division / abs exactly like the oracle, and the update keeps the
reference's multiply-then-subtract (matrixlu.jl:318)."""
import itertools

import numpy as np
import pytest

import oracle_lib as O

pytestmark = pytest.mark.gpu

T = pytest.importorskip("tci_amd")


@pytest.fixture(scope="module")
def ctx():
    c = T.Context(0)
    yield c
    c.close()


def assert_c_bitwise(lu, ref):
    assert lu.npivot == ref.npivot
    assert np.array_equal(lu.rowpermutation - 1, ref.rowpermutation)
    assert np.array_equal(lu.colpermutation - 1, ref.colpermutation)
    assert np.array_equal(lu.L, ref.L)
    assert np.array_equal(lu.U, ref.U)
    assert (lu.error == ref.error) or (np.isnan(lu.error) and np.isnan(ref.error))
    pe = T.pivoterrors(lu)
    assert np.array_equal(pe[:-1], ref.pivoterrors[:-1])


def crand(rng, m, n):
    return rng.random((m, n)) - 0.5 + 1j * (rng.random((m, n)) - 0.5)


@pytest.mark.parametrize("shape,kw", [
    ((7, 5), {}),
    ((30, 40), {}),
    ((100, 80), {"maxrank": 20}),
    ((257, 300), {"maxrank": 64}),
    ((65, 17), {"reltol": 1e-3}),
    ((1, 9), {}),
    ((9, 1), {}),
])
@pytest.mark.parametrize("leftorth", [True, False])
def test_crrlu_random_bitwise(ctx, shape, kw, leftorth):
    A = crand(np.random.default_rng(shape[0] * 7 + shape[1]), *shape)
    lu = T.rrlu(A, leftorthogonal=leftorth, ctx=ctx, **kw)
    ref = O.OracleLUc(A, leftorthogonal=leftorth, **kw)
    assert_c_bitwise(lu, ref)


@pytest.mark.parametrize("leftorth", [True, False])
def test_crrlu_lorentz_ties_bitwise(ctx, leftorth):
    # Pi of the complex Lorentzian coeff / (1 + sum v^2) (test_tensorci2.jl:246-249): values
    # depend on sum v^2 only -> many exact abs2 ties, resolved in column-major order
    d = 6
    I = np.array(list(np.ndindex(d, d))) + 1
    J = np.array(list(np.ndindex(d, d))) + 1
    s = (I ** 2).sum(1)[:, None] + (J ** 2).sum(1)[None, :]
    A = (0.5 - 1.0j) / (s + 1.0)
    for kw in ({}, {"maxrank": 5}, {"reltol": 1e-8}):
        lu = T.rrlu(A, leftorthogonal=leftorth, ctx=ctx, **kw)
        ref = O.OracleLUc(A, leftorthogonal=leftorth, **kw)
        assert_c_bitwise(lu, ref)


@pytest.mark.parametrize("shadow", [1, 0])
@pytest.mark.parametrize("leftorth", [True, False])
def test_crrlu_shadow_search_bitwise(ctx, shadow, leftorth):
    """Sizes the certified shadow search runs on (>= 64 x 64), both settings: ties of a complex
    Lorentzian over 9^2 legs, a rapidly decaying (numerically low-rank) block, NaN-free random
    matrices through two write-back epochs, and an odd row count (shadow padding rows)."""
    ctx.check(ctx.lib.tci_set_c128_shadow(ctx.h, shadow))
    try:
        d = 9
        I = np.array(list(np.ndindex(d, d))) + 1
        s = (I ** 2).sum(1)[:, None] + (I ** 2).sum(1)[None, :]
        cases = [((0.5 - 1.0j) / (s + 1.0), {"maxrank": 30})]
        rng = np.random.default_rng(5)
        U, _ = np.linalg.qr(crand(rng, 160, 160))
        V, _ = np.linalg.qr(crand(rng, 150, 150))
        sv = 2.0 ** -np.arange(150, dtype=float)
        cases.append(((U[:, :150] * sv) @ V.conj().T, {"maxrank": 60, "reltol": 0.0}))
        cases.append((crand(rng, 333, 290), {"maxrank": 40}))
        cases.append((crand(rng, 517, 700) * 1e-30, {"maxrank": 25}))
        for A, kw in cases:
            lu = T.rrlu(A, leftorthogonal=leftorth, ctx=ctx, **kw)
            ref = O.OracleLUc(A, leftorthogonal=leftorth, **kw)
            assert_c_bitwise(lu, ref)
    finally:
        ctx.check(ctx.lib.tci_set_c128_shadow(ctx.h, 1))


def test_crrlu_rank_deficient_and_abstol(ctx):
    rng = np.random.default_rng(3)
    B = crand(rng, 120, 4) @ crand(rng, 4, 90)
    for kw in ({"reltol": 1e-12}, {"abstol": 1e-3}, {"reltol": 0.0, "abstol": 0.0}):
        lu = T.rrlu(B, ctx=ctx, **kw)
        ref = O.OracleLUc(B, **kw)
        assert_c_bitwise(lu, ref)
    assert T.rrlu(B, reltol=1e-12, ctx=ctx).npivot == 4


def test_crrlu_argmax_kat(kats, ctx):
    k = kats["argmax_complex_3x6"]
    Z = np.array(k["re"], float) + 1j * np.array(k["im"], float)
    lu = T.rrlu(Z, maxrank=1, ctx=ctx)
    flat = (np.abs(Z) ** 2).ravel(order="F")
    i = int(np.argmax(flat))
    assert (lu.rowpermutation[0], lu.colpermutation[0]) == (i % 3 + 1, i // 3 + 1)


def test_crrlu_nan_and_empty(ctx):
    A = np.ones((4, 4), complex) + np.eye(4)
    A[2, 0] = complex(np.nan, 0)
    with pytest.raises(O.OracleError, match="lu.L contains NaNs"):
        O.OracleLUc(A)
    with pytest.raises(T.TCIError, match="lu.L contains NaNs"):
        T.rrlu(A, ctx=ctx)
    lu = T.rrlu(np.zeros((0, 5), complex), ctx=ctx)
    assert lu.npivot == 0 and lu.error == 0.0
    # an all-zero matrix: 0/0 in the normalisation -> NaN in L, like the Float64 reference
    Z = np.zeros((6, 4), complex)
    with pytest.raises(O.OracleError, match="lu.L contains NaNs"):
        O.OracleLUc(Z)
    with pytest.raises(T.TCIError, match="lu.L contains NaNs"):
        T.rrlu(Z, ctx=ctx)
    # one row: no normalisation below the pivot, rank 1
    r = np.array([[0.0, 2.0 - 1.0j, 0.5j]])
    assert_c_bitwise(T.rrlu(r, ctx=ctx), O.OracleLUc(r))


def test_crrlu_large_identity(ctx):
    # a size with many workgroups per step; the oracle checks the first pivots bitwise and the
    # factorisation identity covers the rest
    rng = np.random.default_rng(11)
    A = crand(rng, 1500, 1300)
    lu = T.rrlu(A, maxrank=48, ctx=ctx)
    ref = O.OracleLUc(A, maxrank=48)
    assert_c_bitwise(lu, ref)
    P = A[lu.rowpermutation - 1][:, lu.colpermutation - 1]
    k = lu.npivot
    np.testing.assert_allclose(lu.L[:k] @ lu.U[:, :k], P[:k, :k], rtol=0, atol=1e-12)


def test_crrlu_inplace_device_matches_host(ctx):
    import ctypes as C
    rng = np.random.default_rng(21)
    m, n = 300, 260
    A = np.asfortranarray(crand(rng, m, n))
    ref = O.OracleLUc(A, maxrank=40)
    p = C.c_void_p()
    ctx.check(ctx.lib.tci_malloc_d(ctx.h, C.byref(p), A.nbytes))
    try:
        ctx.check(ctx.lib.tci_memcpy_h2d(ctx.h, p, T._lib.ptr(A), A.nbytes))
        rp = np.zeros(m, np.int64)
        cp = np.zeros(n, np.int64)
        pe = np.zeros(41)
        npv, err = C.c_int64(), C.c_double()
        ctx.check(ctx.lib.tci_rrlu_c128_inplace_d(ctx.h, p, m, n, m, 40, 1e-14, 0.0, 1, T._lib.ptr(rp),
                                                  T._lib.ptr(cp), C.byref(npv), C.byref(err),
                                                  T._lib.ptr(pe)))
    finally:
        ctx.lib.tci_free_d(ctx.h, p)
    assert npv.value == ref.npivot
    assert np.array_equal(rp - 1, ref.rowpermutation)
    assert np.array_equal(cp - 1, ref.colpermutation)
    assert err.value == ref.error
    assert np.array_equal(pe, ref.pivoterrors)


@pytest.mark.parametrize("shape,kw", [((30, 24), {"maxrank": 10}), ((30, 24), {}), ((200, 150), {"maxrank": 40}),
                                      ((90, 300), {"reltol": 1e-6})])
@pytest.mark.parametrize("leftorth", [True, False])
def test_cluci_factors_bitwise(ctx, shape, kw, leftorth):
    A = crand(np.random.default_rng(shape[0] + shape[1]), *shape)
    luci = T.MatrixLUCI(A, leftorthogonal=leftorth, ctx=ctx, **kw)
    ri, ci, pe, left, right = O.luci_c128(A, leftorthogonal=leftorth, **kw)
    assert luci.npivots() == len(ri)
    assert np.array_equal(luci.rowindices() - 1, ri)
    assert np.array_equal(luci.colindices() - 1, ci)
    assert np.array_equal(luci.pivoterrors(), pe)
    assert np.array_equal(luci.left(), left)
    assert np.array_equal(luci.right(), right)


# --- ComplexF64 TCI2: the reference's "Lorentz MPS with ValueType=ComplexF64" testset
# (test_tensorci2.jl:246-339, pivotsearch=:full), with nsearchglobalpivot=0. Its
# assertions are properties (rank equality, pivoterror bound, evaluate == f), kept as stated.

def _clorentz(ctx, coeff=0.5 - 1.0j, n=5):
    return T.ComplexScaledEvaluator(coeff, T.lorentz([10] * n, ctx=ctx))


def test_complex_evaluator_values(ctx):
    f = _clorentz(ctx)
    X = np.array([[1, 1, 1, 1, 1], [2, 9, 10, 5, 7], [10, 10, 10, 10, 10]], np.int32)
    v = f.points(X)
    ref = (0.5 - 1.0j) * (1.0 / (1.0 + (X.astype(float) ** 2).sum(1)))
    np.testing.assert_allclose(v, ref, rtol=1e-15)
    Pi, mx = f.pi(X[:, :2], X[:, 2:], 0)
    assert Pi.shape == (3, 3) and mx == pytest.approx(np.abs(Pi).max(), rel=1e-15)


def test_complex_tci2_lorentz(ctx):
    f = _clorentz(ctx)
    tci2, ranks2, errors2 = T.crossinterpolate2(f, [10] * 5, [[1] * 5], tolerance=1e-8, maxiter=8,
                                                sweepstrategy="forward", nsearchglobalpivot=0)
    tci3, ranks3, errors3 = T.crossinterpolate2(f, [10] * 5, [[1] * 5], tolerance=1e-12, maxiter=200,
                                                nsearchglobalpivot=0)
    assert tci3.pivoterror() <= 2e-12
    assert all(d <= 200 for d in tci3.linkdims()) and tci3.rank() <= 200
    for v in itertools.product(range(1, 4), repeat=5):
        val = tci3.evaluate(list(v))
        assert isinstance(val, complex)
        assert val == pytest.approx(f(list(v)), rel=1e-10, abs=1e-14)
    initialpivots = [[1, 1, 1, 1, 1], [10, 8, 10, 4, 4], [5, 4, 8, 9, 3], [7, 7, 10, 5, 9], [7, 7, 10, 5, 9]]
    tci4, _, _ = T.crossinterpolate2(f, [10] * 5, initialpivots, tolerance=1e-12, maxiter=200,
                                     nsearchglobalpivot=0)
    assert tci4.pivoterror() <= 2e-12
    # same function up to a constant factor: the Float64 run finds the same ranks
    fr = T.lorentz([10] * 5, ctx=ctx)
    tr, ranksr, _ = T.crossinterpolate2(fr, [10] * 5, [[1] * 5], tolerance=1e-12, maxiter=200,
                                        nsearchglobalpivot=0)
    assert tci3.rank() == tr.rank()


def test_complex_sitetensor_solve_and_tt_eval(ctx):
    rng = np.random.default_rng(31)
    for r, R in ((1, 5), (7, 70), (40, 400)):
        P = crand(rng, r, r) + 2 * np.eye(r)
        Pi1 = crand(rng, R, r)
        T_ = np.zeros(R * r, np.complex128)
        ctx.check(ctx.lib.tci_sitetensor_solve_c128_h(ctx.h, T._lib.ptr(np.asfortranarray(P)), r,
                                                      T._lib.ptr(np.asfortranarray(Pi1)), R, T._lib.ptr(T_)))
        Tm = T_.reshape((R, r), order="F")
        np.testing.assert_allclose(Tm @ P, Pi1, rtol=0, atol=1e-12)
    # tensor-train evaluation vs the host chain of products (abstracttensortrain.jl:328-342)
    dims, bds = [3, 4, 2, 5], [1, 6, 9, 4, 1]
    cores = [rng.random((bds[t], dims[t], bds[t + 1])) - 0.5 + 1j * rng.random((bds[t], dims[t], bds[t + 1]))
             for t in range(4)]
    tci = T.TensorCI2(dims)
    tci.sitetensors = cores
    X = np.array(list(itertools.product(*[range(1, d + 1) for d in dims])), np.int32)
    got = tci.evaluate_many(X, ctx=ctx)
    ref = np.array([tci.evaluate(list(x)) for x in X])
    np.testing.assert_allclose(got, ref, rtol=1e-13, atol=1e-14)


def test_complex_tci2_with_global_search(ctx):
    # the default flow: site tensors solved every iteration, DefaultGlobalPivotFinder on
    f = _clorentz(ctx)
    tci, ranks, errors = T.crossinterpolate2(f, [10] * 5, [[1] * 5], tolerance=1e-12, maxiter=200,
                                             rng=np.random.default_rng(0))
    assert tci.pivoterror() <= 2e-12
    for v in itertools.product(range(1, 4), repeat=5):
        assert tci.evaluate(list(v)) == pytest.approx(f(list(v)), rel=1e-10, abs=1e-14)


@pytest.mark.parametrize("cplx", [False, True])
def test_cachedfunction_tci2(ctx, cplx):
    # CachedFunction over a device evaluator (misses evaluated in one device batch call, Pi
    # factorised by the device rrLU): same TCI2 result as the evaluator itself; a second run is
    # served from the cache
    base = T.lorentz([10] * 5, ctx=ctx)
    f = _clorentz(ctx) if cplx else base
    cf = T.CachedFunction(f, [10] * 5, complex if cplx else float)
    kw = dict(tolerance=1e-10, maxiter=20, nsearchglobalpivot=0)
    t1, r1, e1 = T.crossinterpolate2(f, [10] * 5, [[1] * 5], **kw)
    t2, r2, e2 = T.crossinterpolate2(cf, [10] * 5, [[1] * 5], **kw)
    assert r1 == r2
    np.testing.assert_allclose(e2, e1, rtol=1e-10, atol=1e-15)
    for b in range(5):
        assert np.array_equal(t1.Iset[b], t2.Iset[b]) and np.array_equal(t1.Jset[b], t2.Jset[b])
    n = cf.ncacheddata()
    assert n > 0
    T.crossinterpolate2(cf, [10] * 5, [[1] * 5], **kw)
    assert cf.ncacheddata() == n
