"""GPU parity: the HIP path (through the C-ABI, via tci_amd) against the CPU oracle.

Bar: bit-exact for rrLU (permutations, L, U, npivot, error) and for the integer-valued integrand
kinds; 1e-12 relative (factors, transcendental integrands) and 1e-10 relative for TCI2 errors, as
stated per test.
"""
import itertools
import os

import numpy as np
import pytest

import oracle_lib as O

# the library's deferred-update depth (tci_abi.cpp tci_ctx::flush_every, env TCI_RRLU_NB), restored
# after tests that change it
LIB_DEFAULT_NB = int(os.environ.get("TCI_RRLU_NB", "10"))
LIB_DEFAULT_EPOCHS = int(os.environ.get("TCI_RRLU_EPOCHS", "0"))  # 0: by shape, the library default

pytestmark = pytest.mark.gpu

T = pytest.importorskip("tci_amd")


@pytest.fixture(scope="module", params=["default", "mid", "pipeline", "pipeline_exact"])
def ctx(request):
    """Every test runs four times: with the default size-based choice of rrLU path (one-workgroup
    LDS kernel for small Pi, persistent grid for mid-size Pi, the pass pipeline above), with the
    mid-size path for everything it fits, and with the pass pipeline forced for every size, with
    the certified fp16 shadow search (default) and without it (every pass reads fp64)."""
    c = T.Context(0)
    c.check(c.lib.tci_set_rrlu_small(c.h, int(request.param == "default")))
    c.check(c.lib.tci_set_rrlu_mid(c.h, int(request.param not in ("pipeline", "pipeline_exact"))))
    c.check(c.lib.tci_set_rrlu_shadow(c.h, int(request.param != "pipeline_exact")))
    yield c
    c.close()


def assert_lu_bitwise(lu, ref):
    assert lu.npivot == ref.npivot
    assert np.array_equal(lu.rowpermutation - 1, ref.rowpermutation)
    assert np.array_equal(lu.colpermutation - 1, ref.colpermutation)
    assert np.array_equal(lu.L, ref.L)
    assert np.array_equal(lu.U, ref.U)
    assert (lu.error == ref.error) or (np.isnan(lu.error) and np.isnan(ref.error))


KAT_MATS = ["rrlu_exact_4x4", "rrlu_truncated_rank1", "rrlu_maxrank4_8x6", "rrlu_identity_pivoterrors",
            "rrlu_limits_5x5", "rrlu_tiny_values"]


@pytest.mark.parametrize("name", KAT_MATS)
@pytest.mark.parametrize("leftorth", [True, False])
def test_rrlu_kats_bitwise(kats, ctx, name, leftorth):
    k = kats[name]
    A = np.array(k["A"], float) * k.get("scale", 1.0)
    kw = dict(k.get("kwargs", {}))
    cases = [c.get("kwargs", {}) for c in k["cases"]] if "cases" in k else [kw]
    for kw in cases:
        lu = T.rrlu(A, leftorthogonal=leftorth, ctx=ctx, **kw)
        ref = O.OracleLU(A, leftorthogonal=leftorth, **kw)
        assert_lu_bitwise(lu, ref)


def test_rrlu_exact_rank3(kats, ctx):
    k = kats["rrlu_exact_rank3"]
    A = np.array(k["p"]) @ np.array(k["q"])
    lu = T.rrlu(A, ctx=ctx)
    assert lu.npivot == 3
    assert_lu_bitwise(lu, O.OracleLU(A))


@pytest.mark.parametrize("m,n,maxrank", [(1, 1, 5), (7, 3, 9), (513, 389, 120), (300, 700, 300),
                                         (1024, 1024, 64)])
@pytest.mark.parametrize("leftorth", [True, False])
def test_rrlu_random_bitwise(ctx, m, n, maxrank, leftorth):
    A = O.fill_uniform(m * n, seed=m * 7 + n).reshape((m, n), order="F")
    lu = T.rrlu(A, maxrank=maxrank, leftorthogonal=leftorth, ctx=ctx)
    assert_lu_bitwise(lu, O.OracleLU(A, maxrank=maxrank, leftorthogonal=leftorth))


@pytest.mark.parametrize("m,n,maxrank", [(8300, 9000, 40), (9000, 8300, 40)])
def test_rrlu_two_staging_groups_bitwise(ctx, m, n, maxrank):
    # 17 row tiles and more than 32 column tiles per workgroup: the pass stages its columns' y's in
    # two groups, and write-back passes race with the second group's staging unless rows outside
    # the trailing block (pivot k's own row) keep their stale values (regression: C5-size Pi)
    A = O.fill_uniform(m * n, seed=m + n).reshape((m, n), order="F")
    lu = T.rrlu(A, maxrank=maxrank, ctx=ctx)
    assert_lu_bitwise(lu, O.OracleLU(A, maxrank=maxrank))


@pytest.mark.parametrize("m,n", [(128, 128), (64, 256), (1, 4000), (4000, 1), (129, 127), (2, 2048)])
def test_rrlu_small_path_limits_bitwise(ctx, m, n):
    # around the single-workgroup limits (m*n <= 16384, m + n <= 4096)
    A = O.fill_uniform(m * n, seed=m + 3 * n).reshape((m, n), order="F")
    for leftorth in (True, False):
        lu = T.rrlu(A, maxrank=min(m, n), leftorthogonal=leftorth, ctx=ctx)
        assert_lu_bitwise(lu, O.OracleLU(A, maxrank=min(m, n), leftorthogonal=leftorth))


def test_rrlu_ties_lorentzian_bitwise(ctx):
    # Lorentzian Pi has many exactly equal entries: exercises the tie order everywhere
    f = O.feval
    I = np.array(list(itertools.product(range(1, 8), repeat=2)), np.int32)
    J = np.array(list(itertools.product(range(1, 8), repeat=2)), np.int32)
    Pi, _ = O.batcheval(1, [1.0], [7] * 4, I, J, 0)
    Pi = Pi[:, 0, :]
    for reltol in (1e-14, 1e-6):
        lu = T.rrlu(Pi, reltol=reltol, ctx=ctx)
        assert_lu_bitwise(lu, O.OracleLU(Pi, reltol=reltol))


def test_rrlu_stop_tests_bitwise(ctx):
    A = O.fill_uniform(200 * 160, seed=3).reshape((200, 160), order="F")
    A = A[:, :40] @ A[:40, :] + 1e-9 * A  # numerically rank ~40
    for kw in ({"reltol": 1e-6}, {"abstol": 1e-5}, {"maxrank": 17}, {"reltol": 0.0, "abstol": 0.0}):
        assert_lu_bitwise(T.rrlu(A, ctx=ctx, **kw), O.OracleLU(A, **kw))


def test_rrlu_nan_raises(ctx):
    # NaN that reaches L (matrixlu.jl:376-378) raises; one that stays outside L/U does not
    A = np.random.default_rng(4).random((5, 5))
    A[3, 0] = np.nan
    with pytest.raises(O.OracleError, match="lu.L contains NaNs"):
        O.OracleLU(A)
    with pytest.raises(T.TCIError, match="lu.L contains NaNs"):
        T.rrlu(A, ctx=ctx)
    B = np.ones((5, 5))
    B[2, 3] = np.nan
    B[0, 0] = 2.0
    assert_lu_bitwise(T.rrlu(B, ctx=ctx), O.OracleLU(B))


def test_rrlu_empty(ctx):
    lu = T.rrlu(np.zeros((0, 4)), ctx=ctx)
    assert lu.npivot == 0 and lu.error == 0.0


@pytest.mark.parametrize("leftorth", [True, False])
def test_luci_factors(ctx, kats, leftorth):
    for A in (np.array(kats["luci_maxrank4_8x6"]["A"]),
              O.fill_uniform(300 * 200, 11).reshape((300, 200), order="F")):
        for maxrank in (4, 50, 1000):
            luci = T.MatrixLUCI(A, maxrank=maxrank, leftorthogonal=leftorth, ctx=ctx)
            ref = O.OracleLU(A, maxrank=maxrank, leftorthogonal=leftorth)
            assert np.array_equal(luci.rowindices() - 1, ref.rowindices())
            assert np.array_equal(luci.colindices() - 1, ref.colindices())
            assert np.array_equal(luci.pivoterrors(), ref.pivoterrors)
            np.testing.assert_allclose(luci.left(), ref.left, rtol=1e-12, atol=1e-12 * np.abs(ref.left).max())
            np.testing.assert_allclose(luci.right(), ref.right, rtol=1e-12, atol=1e-12 * np.abs(ref.right).max())


@pytest.mark.parametrize("leftorth", [True, False])
def test_luci_factors_large_rank(ctx, leftorth):
    # np beyond 512: the blocked triangular solves with 16 (np <= 1024) and 8 right-hand sides
    A = O.fill_uniform(1400 * 1200, 12).reshape((1400, 1200), order="F")
    for maxrank in (700, 1100):
        luci = T.MatrixLUCI(A, maxrank=maxrank, leftorthogonal=leftorth, ctx=ctx)
        ref = O.OracleLU(A, maxrank=maxrank, leftorthogonal=leftorth)
        assert np.array_equal(luci.rowindices() - 1, ref.rowindices())
        assert np.array_equal(luci.colindices() - 1, ref.colindices())
        np.testing.assert_allclose(luci.left(), ref.left, rtol=1e-12, atol=1e-12 * np.abs(ref.left).max())
        np.testing.assert_allclose(luci.right(), ref.right, rtol=1e-12, atol=1e-12 * np.abs(ref.right).max())


KINDS = [
    (O_SUM := 0, [], [3, 4, 2, 5, 3]),
    (1, [1.0], [10] * 6),
    (1, [0.5], [7] * 5),
    (2, None, [3, 4, 2, 5]),
    (3, [1.0 / 64, 8.5], [16] * 6),
    (5, [10.0, 2 * np.pi * 100, 1.1], [2] * 20),
    (6, [1.0, 1.0, 1e-4, 2.0], [2] * 12),
    (4, None, [6] * 8),           # GAUSSMIX: rank-K MFMA GEMM path
    (8, None, [5, 3, 4, 5, 2, 5]),  # CP-rank-K synthetic: rank-K MFMA GEMM path
]


def _random_params(kind, ld, rng, K=37):
    L = len(ld)
    if kind == 2:
        return rng.random(int(np.prod(ld))).tolist()
    if kind == 4:  # K Gaussians, mixed-sign weights
        return np.concatenate([[K, 0.07], rng.random(K * L) * max(ld), rng.random(K) - 0.3]).tolist()
    if kind == 8:
        dmax = max(ld)
        return np.concatenate([[K, dmax], rng.random(K * L * dmax) * 1.5]).tolist()
    return None


@pytest.mark.parametrize("kind,params,ld", KINDS)
@pytest.mark.parametrize("M", [0, 1])
def test_batcheval_vs_oracle(ctx, kind, params, ld, M):
    rng = np.random.default_rng(kind * 10 + M)
    if params is None:
        params = _random_params(kind, ld, rng)
    L = len(ld)
    nl = L // 2 - (1 if M else 0)
    nr = L - nl - M
    I = np.stack([rng.integers(1, ld[t] + 1, 37) for t in range(nl)], axis=1).astype(np.int32) if nl else np.zeros((37, 0), np.int32)
    J = np.stack([rng.integers(1, ld[nl + M + t] + 1, 29) for t in range(nr)], axis=1).astype(np.int32)
    ref, rmx = O.batcheval(kind, params, ld, I, J, M)
    f = T.GPUBatchEvaluator(kind, params, ld, ctx=ctx)
    got = f.batch([list(r) for r in I] if nl else [[] for _ in range(37)], [list(r) for r in J], M)
    ref = ref.reshape(got.shape, order="F")
    if kind in (0, 1, 2):
        assert np.array_equal(got, ref)  # integer-exact kinds: bitwise
        _, gmx = f.pi(I, J, M)
        assert gmx == rmx
    else:
        # ocml vs glibc exp/sin/pow: a few ulp of the largest intermediate; separable kinds (4, 8)
        # also split the exponential / product and sum the K terms in MFMA order
        np.testing.assert_allclose(got, ref, rtol=1e-12, atol=1e-13 * np.abs(ref).max())
        _, gmx = f.pi(I, J, M)
        assert gmx == pytest.approx(rmx, rel=1e-13)


def test_batcheval_tt_and_gaussmix(ctx):
    rng = np.random.default_rng(5)
    ld = [2, 3, 3, 2]
    bd = [1, 2, 3, 2, 1]
    cores = [rng.random((bd[p], ld[p], bd[p + 1])) for p in range(4)]
    f = T.tensortrain_function(cores, ctx=ctx)
    params = np.concatenate([np.array(bd, float)] + [c.ravel(order="F") for c in cores])
    X = np.array(list(itertools.product(*[range(1, d + 1) for d in ld])), np.int32)
    got = f.points(X)
    ref = np.array([O.feval(7, params, ld, x) for x in X])
    np.testing.assert_allclose(got, ref, rtol=1e-13)
    cen = rng.random((4, 5)) * 6
    g = T.gaussmix([6] * 5, 0.1, cen, [1.0, -0.5, 0.25, 2.0], ctx=ctx)
    p2 = np.concatenate([[4, 0.1], cen.ravel(), [1.0, -0.5, 0.25, 2.0]])
    X = rng.integers(1, 7, (50, 5)).astype(np.int32)
    ref = np.array([O.feval(4, p2, [6] * 5, x) for x in X])
    np.testing.assert_allclose(g.points(X), ref, rtol=1e-12, atol=1e-13 * np.abs(ref).max())


@pytest.mark.parametrize("shape", [(1, 1, 1), (130, 70, 5), (200, 257, 64), (64, 64, 1024)])
def test_cp_gemm_sizes(ctx, shape):
    # rank-K GEMM assembly across tile edges (R, n not multiples of 64; K not a multiple of 4)
    m, n, K = shape
    rng = np.random.default_rng(m + n + K)
    ld = [4, 3, 5, 4]
    params = np.concatenate([[K, 5], rng.random(K * 4 * 5) - 0.5])
    I = np.stack([rng.integers(1, ld[t] + 1, m) for t in range(2)], axis=1).astype(np.int32)
    J = np.stack([rng.integers(1, ld[2 + t] + 1, n) for t in range(2)], axis=1).astype(np.int32)
    ref, rmx = O.batcheval(8, params, ld, I, J, 0)
    f = T.GPUBatchEvaluator(8, params, ld, ctx=ctx)
    got, gmx = f.pi(I, J, 0)
    ref = ref.reshape(got.shape, order="F")
    np.testing.assert_allclose(got, ref, rtol=1e-12, atol=1e-13 * np.abs(ref).max())
    assert gmx == pytest.approx(rmx, rel=1e-12)


def test_sitetensor_solve(ctx):
    rng = np.random.default_rng(9)
    M = rng.random((12, 12))
    f = T.table(M, ctx=ctx)
    tci, ranks, errors = T.crossinterpolate2(f, maxbonddim=6, nsearchglobalpivot=0)
    Ib, Jb, Inext = tci.Iset[0], tci.Jset[0], tci.Iset[1]
    tens = tci.setsitetensor(f, 1)
    P = M[np.ix_(Inext[:, 0] - 1, Jb[:, 0] - 1)]
    Pi1 = M[:, Jb[:, 0] - 1]
    ref = O.sitetensor_solve(P, Pi1)
    np.testing.assert_allclose(tens.reshape(ref.shape, order="F"), ref, rtol=1e-10, atol=1e-12)


@pytest.mark.parametrize("r,R", [(100, 1000), (300, 777), (600, 1201)])
def test_sitetensor_solve_blocked(ctx, r, R):
    # T = Pi1 * P^-1 (tensorci2.jl:620-627) with the LDS-blocked getrs (32 / 16 / 8 right-hand
    # sides per workgroup, partial tiles included)
    import ctypes as C
    rng = np.random.default_rng(r + R)
    P = rng.random((r, r)) + r * np.eye(r) * rng.choice([-1, 1], r)
    Pi1 = rng.random((R, r))
    T_ = np.zeros(R * r)
    ctx.check(ctx.lib.tci_sitetensor_solve_h(ctx.h, T._lib.ptr(np.asfortranarray(P).ravel(order="F")), r,
                                             T._lib.ptr(np.asfortranarray(Pi1).ravel(order="F")), R,
                                             T._lib.ptr(T_)))
    ref = O.sitetensor_solve(P, Pi1)
    got = T_.reshape((R, r), order="F")
    np.testing.assert_allclose(got, ref.reshape(got.shape, order="F"), rtol=1e-10, atol=1e-12 * np.abs(ref).max())


# ------------------------------------------------------------------ TCI2
def _compare_tci(tci, ranks, errors, rt, rranks, rerrors, rtol=1e-10, exact_f=True):
    """exact_f: integer-exact integrand (bitwise Pi) -> errors to 1e-10 relative of themselves;
    transcendental integrands (ocml vs glibc ulps in Pi) -> errors, which are already relative to
    maxsamplevalue, to 1e-10 absolute (i.e. 1e-10 relative to the function scale)."""
    assert ranks == rranks
    if exact_f:
        np.testing.assert_allclose(errors, rerrors, rtol=rtol, atol=0)
    else:
        np.testing.assert_allclose(errors, rerrors, rtol=0, atol=rtol)
    for p in range(len(tci.localdims)):
        assert np.array_equal(tci.Iset[p], rt.Iset(p)), p
        assert np.array_equal(tci.Jset[p], rt.Jset(p)), p
    if exact_f:
        np.testing.assert_allclose(tci.pivoterrors, rt.pivoterrors, rtol=rtol, atol=0)
    else:
        np.testing.assert_allclose(tci.pivoterrors, rt.pivoterrors, rtol=0, atol=rtol * rt.maxsamplevalue)
    if exact_f:
        assert tci.maxsamplevalue == rt.maxsamplevalue
    else:
        assert tci.maxsamplevalue == pytest.approx(rt.maxsamplevalue, rel=1e-13)
    if exact_f:
        for p in range(len(tci.localdims)):
            ref = rt.sitetensor(p)
            np.testing.assert_allclose(tci.sitetensors[p], ref, rtol=1e-9, atol=1e-12 * max(1.0, np.abs(ref).max()))
    else:
        # ulp differences in Pi are amplified by cond(pivot block) in the factors; the parity
        # quantity is the interpolated value: within 1e-9 of maxsamplevalue on random points
        rng = np.random.default_rng(0)
        X = np.stack([rng.integers(1, d + 1, 300) for d in tci.localdims], axis=1)
        got = tci.evaluate_many(X)
        ref = np.array([rt.evaluate(list(x)) for x in X])
        np.testing.assert_allclose(got, ref, rtol=0, atol=1e-9 * rt.maxsamplevalue)


@pytest.mark.parametrize("bd", [[1, 3, 1], [1, 5, 70, 9, 1], [1, 130, 260, 4, 1]])
def test_tt_evaluate_many_vs_oracle(ctx, bd):
    # batched tensor-train evaluation (global pivot search) vs the oracle's evaluate chain
    rng = np.random.default_rng(len(bd) + bd[1])
    L = len(bd) - 1
    ld = [3, 4, 2, 5][:L]
    cores = [rng.random((bd[p], ld[p], bd[p + 1])) - 0.5 for p in range(L)]
    tci = T.TensorCI2(ld)
    tci.sitetensors = cores
    X = np.stack([rng.integers(1, d + 1, 257) for d in ld], axis=1).astype(np.int32)
    got = tci.evaluate_many(X, ctx=ctx)
    params = np.concatenate([np.array(bd, float)] + [c.ravel(order="F") for c in cores])
    ref = np.array([O.feval(7, params, ld, x) for x in X])
    np.testing.assert_allclose(got, ref, rtol=1e-12, atol=1e-13 * np.abs(ref).max())


def test_tci2_pivoterrors_kat(kats, ctx):
    k = kats["tci2_pivoterrors"]
    M = np.diag(k["diags"])
    f = T.table(M, ctx=ctx)
    tci, ranks, errors = T.crossinterpolate2(f, initialpivots=k["initialpivots"], tolerance=k["tolerance"],
                                             nsearchglobalpivot=0)
    assert list(tci.pivoterrors) == k["expect"]["pivoterrors"]


def test_tci2_lorentz5d_kat(kats, ctx):
    k = kats["tci2_lorentz5d"]
    n, d = k["n"], k["d"]
    f = T.lorentz([d] * n, ctx=ctx)
    tci = T.TensorCI2.from_function(f, [d] * n)
    assert tci.linkdims() == [1] * (n - 1)
    for b in range(1, n):
        tci.updatepivots(b, f, True, reltol=1e-8, maxbonddim=2)
    assert tci.linkdims() == k["updatepivots_maxbonddim2"]["expect_linkdims"]
    tci.addglobalpivots1sitesweep(f, [k["globalpivot"]], reltol=1e-12)
    assert tci.linkdims() == k["after_global_1site"]["expect_linkdims"]
    # same sequence on the oracle: identical sets and tensors
    rt = O.OracleTCI2(1, [1.0], [d] * n)
    for b in range(n - 1):
        rt.updatepivots(b, True, 1e-8, 0.0, 2)
    rt.addglobalpivots([k["globalpivot"]])
    rt.makecanonical(reltol=1e-12)
    for p in range(n):
        assert np.array_equal(tci.Iset[p], rt.Iset(p)) and np.array_equal(tci.Jset[p], rt.Jset(p))
        np.testing.assert_allclose(tci.sitetensors[p], rt.sitetensor(p), rtol=1e-9, atol=1e-14)
    tci3, ranks, errors = T.crossinterpolate2(f, tolerance=1e-12, maxiter=200, nsearchglobalpivot=0)
    assert tci3.pivoterror() <= 2e-12
    for v in itertools.product(range(1, 4), repeat=n):
        assert tci3.evaluate(v) == pytest.approx(1.0 / (sum(x * x for x in v) + 1), rel=1.5e-8)


@pytest.mark.parametrize("strategy", ["backandforth", "forward"])
@pytest.mark.parametrize("strict", [False, True])
def test_tci2_lorentz_vs_oracle(ctx, strategy, strict):
    ld = [10] * 6
    f = T.lorentz(ld, ctx=ctx)
    kw = dict(tolerance=1e-10, maxiter=10, sweepstrategy=strategy, strictlynested=strict)
    tci, ranks, errors = T.crossinterpolate2(f, nsearchglobalpivot=0, **kw)
    rt, rranks, rerrors = O.crossinterpolate2(1, [1.0], ld, **kw)
    _compare_tci(tci, ranks, errors, rt, rranks, rerrors)


def test_tci2_config1_readme_lorentzian(ctx):
    """BASELINE config 1: f(v) = 1/(1+v'v), localdims = fill(10, 8), tol = 1e-8."""
    ld = [10] * 8
    f = T.lorentz(ld, ctx=ctx)
    tci, ranks, errors = T.crossinterpolate2(f, tolerance=1e-8, nsearchglobalpivot=0)
    rt, rranks, rerrors = O.crossinterpolate2(1, [1.0], ld, tolerance=1e-8)
    _compare_tci(tci, ranks, errors, rt, rranks, rerrors)


def test_tci2_quantics_and_gauss_vs_oracle(ctx):
    for kind, params, ld, kw in (
        (5, [10.0, 2 * np.pi * 100, 1.1], [2] * 12, dict(tolerance=1e-10, maxbonddim=40, maxiter=8)),
        (6, [1.0, 1.0, 1e-4, 2.0], [2] * 10, dict(tolerance=1e-12, maxiter=6)),
        (3, [1.0 / 64, 8.5], [16] * 6, dict(tolerance=1e-10, maxbonddim=64, maxiter=6)),
    ):
        f = T.GPUBatchEvaluator(kind, params, ld, ctx=ctx)
        piv = [T.optfirstpivot(f, ld, [1] * len(ld))]  # f(1,...,1) = 0 for the oscillatory kind
        tci, ranks, errors = T.crossinterpolate2(f, initialpivots=piv, nsearchglobalpivot=0, **kw)
        rt, rranks, rerrors = O.crossinterpolate2(kind, params, ld, piv, **kw)
        _compare_tci(tci, ranks, errors, rt, rranks, rerrors, exact_f=False)


def test_tci2_tt_function_reconstruction(ctx):
    rng = np.random.default_rng(7)
    ld = [2, 3, 3, 2]
    bd = [1, 2, 3, 2, 1]
    cores = [rng.random((bd[p], ld[p], bd[p + 1])) for p in range(4)]
    f = T.tensortrain_function(cores, ctx=ctx)
    tci, ranks, errors = T.crossinterpolate2(f, tolerance=1e-10, maxbonddim=10, nsearchglobalpivot=0)
    X = np.array(list(itertools.product(*[range(1, d + 1) for d in ld])))
    np.testing.assert_allclose(tci.evaluate_many(X), f.points(X), rtol=1e-8)


def test_tci2_default_global_search_runs(ctx):
    """Default nsearchglobalpivot=5 (random search; statistical parity only)."""
    f = T.quantics_osc(10, ctx=ctx)
    rng = np.random.default_rng(1234)
    first = T.optfirstpivot(f, [2] * 10, list(rng.integers(1, 3, 10)))
    tci, ranks, errors = T.crossinterpolate2(f, initialpivots=[first], tolerance=1e-12, maxbonddim=100,
                                             maxiter=100, nsearchglobalpivot=10, rng=rng)
    assert errors[-1] < 1e-10


def test_optfirstpivot_matches_restatement(ctx):
    """optfirstpivot (util.jl:260-298) batched per leg on the GPU == sequential restatement."""
    ld = [2] * 12
    params = [10.0, 2 * np.pi * 100, 1.1]
    f = T.quantics_osc(12, ctx=ctx)
    start = [1, 2] * 6
    got = T.optfirstpivot(f, ld, start)
    pivot = list(start)
    valf = abs(O.feval(5, params, ld, pivot))
    for _ in range(1000):
        prev = valf
        for i in range(len(ld)):
            for d in range(1, ld[i] + 1):
                bak = pivot[i]
                pivot[i] = d
                nv = abs(O.feval(5, params, ld, pivot))
                if nv > valf:
                    valf = nv
                else:
                    pivot[i] = bak
        if prev == valf:
            break
    assert got == pivot


@pytest.mark.parametrize("nb", [1, 2, 3, 8, 16])
def test_rrlu_deferred_depth_bitwise(ctx, nb):
    """The deferred-update depth changes only the schedule: every nb gives the reference's bits."""
    ctx.check(ctx.lib.tci_set_rrlu_flush(ctx.h, nb))
    try:
        A = O.fill_uniform(1000 * 700, seed=nb).reshape((1000, 700), order="F")
        for lo in (True, False):
            assert_lu_bitwise(T.rrlu(A, maxrank=150, leftorthogonal=lo, ctx=ctx),
                              O.OracleLU(A, maxrank=150, leftorthogonal=lo))
        I = np.array(list(itertools.product(range(1, 8), repeat=2)), np.int32)
        Pi, _ = O.batcheval(1, [1.0], [7] * 4, I, I, 0)
        Pi = Pi[:, 0, :]
        assert_lu_bitwise(T.rrlu(Pi, ctx=ctx), O.OracleLU(Pi))
        B = A[:300, :40] @ A[:40, :250] + 1e-10 * A[:300, :250]
        for kw in ({"reltol": 1e-7}, {"abstol": 1e-6}):
            assert_lu_bitwise(T.rrlu(B, ctx=ctx, **kw), O.OracleLU(B, **kw))
    finally:
        ctx.check(ctx.lib.tci_set_rrlu_flush(ctx.h, LIB_DEFAULT_NB))
