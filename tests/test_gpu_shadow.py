"""GPU parity of the certified fp16 shadow search (k_pass_mf, DESIGN.md K2, with its two-level epoch of
refreshes and deep exact passes k_pass_x): the pass pipeline with
the shadow on must give the reference's bits (oracle) on inputs chosen to stress the certificate:
massive ties, exact zeros after the rank, rapidly decaying pivots (the kernel falls back to the
exact body pass by pass), magnitudes where fp32 would underflow or overflow, NaN and Inf entries,
odd shapes and every deferred depth. Each case runs with the shadow search on and off.
"""
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


@pytest.fixture(scope="module", params=["shadow", "exact"])
def pctx(request):
    """The pass pipeline forced for every size, with and without the shadow search."""
    c = T.Context(0)
    c.check(c.lib.tci_set_rrlu_small(c.h, 0))
    c.check(c.lib.tci_set_rrlu_mid(c.h, 0))
    c.check(c.lib.tci_set_rrlu_shadow(c.h, int(request.param == "shadow")))
    yield c
    c.close()


def outcome_gpu(A, ctx, **kw):
    try:
        return T.rrlu(A, ctx=ctx, **kw)
    except T.TCIError as e:
        return ("error", str(e))


def outcome_ref(A, **kw):
    try:
        return O.OracleLU(A, **kw)
    except O.OracleError as e:
        return ("error", str(e))


def assert_same(got, ref):
    if isinstance(ref, tuple):
        assert isinstance(got, tuple), "oracle raised, device did not"
        assert ref[1] in got[1] or got[1] in ref[1], (got, ref)
        return
    assert not isinstance(got, tuple), got
    assert got.npivot == ref.npivot
    assert np.array_equal(got.rowpermutation - 1, ref.rowpermutation)
    assert np.array_equal(got.colpermutation - 1, ref.colpermutation)
    assert np.array_equal(got.L, ref.L, equal_nan=True)
    assert np.array_equal(got.U, ref.U, equal_nan=True)
    assert (got.error == ref.error) or (np.isnan(got.error) and np.isnan(ref.error))


def rand(m, n, seed):
    return O.fill_uniform(m * n, seed=seed).reshape((m, n), order="F")


@pytest.mark.parametrize("nb,epochs", [(2, 1), (10, 1), (16, 1), (2, 4), (3, 10), (5, 6), (8, 4), (10, 3),
                                       (15, 2)])
@pytest.mark.parametrize("leftorth", [True, False])
def test_shadow_random(pctx, nb, epochs, leftorth):
    """Every schedule of the two-level epoch: shadow epochs of nb pivots, a refresh
    of the shadow by the MFMA search after each, an fp64 write-back after every epochs-th (exact
    pending updates up to nb * epochs, x's in LDS from 12 on) -- the reference's bits each time."""
    pctx.check(pctx.lib.tci_set_rrlu_flush(pctx.h, nb))
    pctx.check(pctx.lib.tci_set_rrlu_epochs(pctx.h, epochs))
    try:
        A = rand(1100, 900, 11 + nb + 100 * epochs)
        kw = dict(maxrank=180, leftorthogonal=leftorth)
        assert_same(outcome_gpu(A, pctx, **kw), outcome_ref(A, **kw))
    finally:
        pctx.check(pctx.lib.tci_set_rrlu_flush(pctx.h, LIB_DEFAULT_NB))
        pctx.check(pctx.lib.tci_set_rrlu_epochs(pctx.h, LIB_DEFAULT_EPOCHS))


@pytest.mark.parametrize("epochs", [2, 3])
def test_shadow_refresh_fallbacks(pctx, epochs):
    """Decays at which the refresh's accumulated bound stops certifying part of the way through an
    exact epoch: refreshes then rewrite the shadow from exact values (k_pass_x mode 2), later read
    passes of the same epoch run k_pass_x's exact body with up to nb * epochs pending updates."""
    rng = np.random.default_rng(epochs)
    pctx.check(pctx.lib.tci_set_rrlu_epochs(pctx.h, epochs))
    try:
        for base in (1.05, 1.2, 1.6):
            Q1 = rng.standard_normal((900, 200))
            Q2 = rng.standard_normal((200, 800))
            A = (Q1 * base ** -np.arange(200.0)) @ Q2
            for lo in (True, False):
                kw = dict(maxrank=150, reltol=0.0, leftorthogonal=lo)
                assert_same(outcome_gpu(A, pctx, **kw), outcome_ref(A, **kw))
    finally:
        pctx.check(pctx.lib.tci_set_rrlu_epochs(pctx.h, LIB_DEFAULT_EPOCHS))


@pytest.mark.parametrize("scale", [1e-300, 1e-45, 1e-36, 1e-30, 1e25, 1e31, 1e40, 1e150, 1e300])
def test_shadow_magnitudes(pctx, scale):
    """fp32 underflow / overflow regions: the certificate's absolute term and the overflow guard
    switch the kernel to its exact body; in between the shadow stays on."""
    A = rand(700, 650, 5) * scale
    kw = dict(maxrank=90)
    assert_same(outcome_gpu(A, pctx, **kw), outcome_ref(A, **kw))


def test_shadow_lorentzian_ties(pctx):
    """A Pi matrix of the Lorentzian over integer legs: every value depends only on a sum of
    squares, so the maximum is attained many times and the tie order decides every pivot."""
    import itertools
    I = np.array(list(itertools.product(range(1, 8), repeat=3)), np.int32)
    Pi, _ = O.batcheval(1, [1.0], [7] * 6, I, I, 0)
    Pi = np.ascontiguousarray(Pi[:, 0, :])
    for lo in (True, False):
        kw = dict(maxrank=60, leftorthogonal=lo, reltol=0.0)
        assert_same(outcome_gpu(Pi, pctx, **kw), outcome_ref(Pi, **kw))


def test_shadow_integer_pattern_ties(pctx):
    i = np.arange(1, 1001)[:, None]
    j = np.arange(1, 801)[None, :]
    A = ((i * j) % 7 - 3).astype(np.float64)
    kw = dict(maxrank=40, reltol=0.0)
    assert_same(outcome_gpu(A, pctx, **kw), outcome_ref(A, **kw))


def test_shadow_constant_and_exact_low_rank(pctx):
    C = np.ones((600, 500))
    assert_same(outcome_gpu(C, pctx, maxrank=50), outcome_ref(C, maxrank=50))
    B = rand(800, 30, 7) @ rand(30, 760, 8)  # exact rank 30; past it only roundoff (or zeros)
    for kw in (dict(maxrank=60, reltol=0.0), dict(maxrank=60)):
        assert_same(outcome_gpu(B, pctx, **kw), outcome_ref(B, **kw))


def test_shadow_geometric_decay(pctx):
    """Pivots decay by 2 (and by 10) per step: the certificate is loose relative to the current
    maximum after a few pending updates, and the kernel must fall back to its exact body."""
    rng = np.random.default_rng(2)
    for base in (2.0, 10.0):
        Q1 = rng.standard_normal((700, 120))
        Q2 = rng.standard_normal((120, 640))
        A = (Q1 * base ** -np.arange(120.0)) @ Q2
        kw = dict(maxrank=110, reltol=0.0)
        assert_same(outcome_gpu(A, pctx, **kw), outcome_ref(A, **kw))


def test_shadow_nan_inf(pctx):
    A = rand(900, 700, 9)
    B = A.copy()
    B[5, :] = np.nan  # a NaN row: never selected, becomes part of L -> raises like the reference
    assert_same(outcome_gpu(B, pctx, maxrank=40), outcome_ref(B, maxrank=40))
    C = A.copy()
    C[:, 17] = np.nan
    C[33, 17] = 5.0
    assert_same(outcome_gpu(C, pctx, maxrank=40), outcome_ref(C, maxrank=40))
    D = A.copy()
    D[100, 200] = np.inf
    assert_same(outcome_gpu(D, pctx, maxrank=40), outcome_ref(D, maxrank=40))
    E = A.copy()
    E[300:305, 40] = 1e38  # fp32-overflowing values in an otherwise benign matrix
    assert_same(outcome_gpu(E, pctx, maxrank=40), outcome_ref(E, maxrank=40))


@pytest.mark.parametrize("m,n", [(1023, 777), (513, 1029), (4097, 300), (300, 4097)])
def test_shadow_odd_shapes(pctx, m, n):
    A = rand(m, n, m + n)
    for lo in (True, False):
        kw = dict(maxrank=70, leftorthogonal=lo)
        assert_same(outcome_gpu(A, pctx, **kw), outcome_ref(A, **kw))


def test_shadow_inplace_device_odd_lda(pctx):
    """tci_rrlu_inplace_d with a leading dimension that is not a multiple of 4 runs the exact
    passes (the 16-B four-row loads need lda % 4 == 0) -- same bits either way."""
    import ctypes as C

    m, n, lda = 601, 500, 606
    A = rand(lda, n, 21)
    A[m:, :] = 0.0
    L = pctx.lib
    ptr = C.c_void_p()
    pctx.check(L.tci_malloc_d(pctx.h, C.byref(ptr), A.size * 8))
    try:
        Af = np.asfortranarray(A)
        pctx.check(L.tci_memcpy_h2d(pctx.h, ptr, Af.ctypes.data, A.size * 8))
        rowp = np.zeros(m, np.int64)
        colp = np.zeros(n, np.int64)
        npiv = C.c_int64()
        err = C.c_double()
        pctx.check(L.tci_rrlu_inplace_d(pctx.h, ptr, m, n, lda, 60, 1e-14, 0.0, 1, rowp.ctypes.data,
                                        colp.ctypes.data, C.byref(npiv), C.byref(err), None))
        ref = O.OracleLU(np.ascontiguousarray(A[:m, :]), maxrank=60)
        assert npiv.value == ref.npivot
        assert np.array_equal(rowp - 1, ref.rowpermutation)
        assert np.array_equal(colp - 1, ref.colpermutation)
        assert err.value == ref.error
    finally:
        pctx.check(L.tci_free_d(pctx.h, ptr))
