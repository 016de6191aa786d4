"""GPU parity of the persistent shadow-epoch launch (tci_rrlu.hip k_pass_mf_epoch):
the read-only passes of a shadow epoch in one launch whose resident grid hands each commit of
_optimizerrlu!'s loop (matrixlu.jl:356-369) to the next pass in place of a kernel boundary. Results
must be the reference's bits (oracle) whatever the schedule, and equal to the per-pass launches':
every depth nb and exact-epoch length, both orientations, a stop test inside an epoch, NaN entries,
a certificate that fails mid-epoch (the launch ends, the host resumes with per-pass launches), and a
grid that is NOT co-resident (test mode: the launch gives up and the factorisation resumes).
"""
import os

import numpy as np
import pytest

import oracle_lib as O

pytestmark = pytest.mark.gpu

T = pytest.importorskip("tci_amd")

EPOCH_FAMS = (41, 42)  # tci_hip.h tci_last_kernel_units: persistent launches (first shadow epoch / EXT)


def rand(m, n, seed):
    return O.fill_uniform(m * n, seed=seed).reshape((m, n), order="F")


NOT_BUILT = "persistent epoch grid not built (the default build; make variant VFLAGS=-DTCI_EPOCH_GRID=1)"


def make_ctx(persist=1):
    c = T.Context(0)
    c.check(c.lib.tci_set_rrlu_small(c.h, 0))
    c.check(c.lib.tci_set_rrlu_mid(c.h, 0))
    rc = c.lib.tci_set_rrlu_persist(c.h, persist)
    if rc != 0 and persist:
        c.close()
        pytest.skip(NOT_BUILT)
    c.check(rc)
    return c


def test_default_build_refuses_persist():
    """The grid was measured slower and is compiled only on request: a build
    without it refuses tci_set_rrlu_persist(ctx, 1 | 2) with TCI_ERR_ARG, and 0 is always accepted."""
    c = T.Context(0)
    try:
        assert c.lib.tci_set_rrlu_persist(c.h, 0) == 0
        rc = c.lib.tci_set_rrlu_persist(c.h, 1)
        if rc != 0:
            assert rc == 1  # TCI_ERR_ARG
            assert "TCI_EPOCH_GRID" in c.lib.tci_last_error(c.h).decode()
    finally:
        c.close()


@pytest.fixture(scope="module")
def pctx():
    c = make_ctx()
    yield c
    c.close()


def assert_same(got, ref):
    assert got.npivot == ref.npivot
    assert np.array_equal(got.rowpermutation - 1, ref.rowpermutation)
    assert np.array_equal(got.colpermutation - 1, ref.colpermutation)
    assert np.array_equal(got.L, ref.L, equal_nan=True)
    assert np.array_equal(got.U, ref.U, equal_nan=True)
    assert (got.error == ref.error) or (np.isnan(got.error) and np.isnan(ref.error))


def epoch_passes(ctx):
    """passes the persistent launches of the last factorisation covered (timing on: every 3rd launch)"""
    return sum(ctx.kernel_units(f)[2] for f in EPOCH_FAMS)


def run(ctx, A, **kw):
    ctx.set_timing(True, stride=1)
    try:
        lu = T.rrlu(A, ctx=ctx, **kw)
        return lu, epoch_passes(ctx)
    finally:
        ctx.set_timing(False)


@pytest.mark.parametrize("nb,epochs", [(10, 1), (10, 3), (4, 5), (11, 2), (12, 2), (2, 8)])
@pytest.mark.parametrize("leftorth", [True, False])
def test_persist_bitwise(pctx, nb, epochs, leftorth):
    """Every schedule: runs of nb - 1 read-only passes per launch (nb = 12: passes of depth 11 run
    per pass, the run before them persistent), first and later shadow epochs (EXT) of an exact
    epoch of nb x epochs pivots -- the oracle's bits, and the persistent form actually ran."""
    pctx.check(pctx.lib.tci_set_rrlu_flush(pctx.h, nb))
    pctx.check(pctx.lib.tci_set_rrlu_epochs(pctx.h, epochs))
    try:
        A = rand(2100, 1900, 7 + nb + 10 * epochs)
        kw = dict(maxrank=150, leftorthogonal=leftorth)
        got, npers = run(pctx, A, **kw)
        assert_same(got, O.OracleLU(A, **kw))
        if nb > 2:
            assert npers > 0, "no persistent launch ran"
        assert pctx.lib.tci_rrlu_persist_faulted(pctx.h) == 0
    finally:
        pctx.check(pctx.lib.tci_set_rrlu_flush(pctx.h, 10))
        pctx.check(pctx.lib.tci_set_rrlu_epochs(pctx.h, 0))


def test_persist_equals_per_pass():
    """The same factorisation with the persistent launch on and off: identical bits (the pass
    bodies are the same; only the hand-off between passes differs)."""
    A = rand(4100, 4000, 3)
    res = []
    for persist in (1, 0):
        c = make_ctx(persist)
        try:
            c.check(c.lib.tci_set_rrlu_epochs(c.h, 3))
            lu = T.rrlu(A, ctx=c, maxrank=200)
            res.append((lu.npivot, lu.rowpermutation.copy(), lu.colpermutation.copy(), lu.L.copy(), lu.U.copy(),
                        lu.error))
        finally:
            c.close()
    a, b = res
    assert a[0] == b[0] == 200
    for x, y in zip(a[1:5], b[1:5]):
        assert np.array_equal(x, y)
    assert a[5] == b[5]


def test_persist_stop_inside_epoch(pctx):
    """A rank-37 matrix factorised to maxrank 120: the stop test (matrixlu.jl:359-368) fires in a
    pass of a persistent launch; every workgroup sees it in the next pass and the launch ends."""
    rng = np.random.default_rng(5)
    A = rng.standard_normal((1500, 37)) @ rng.standard_normal((37, 1300))
    for kw in (dict(maxrank=120), dict(maxrank=120, reltol=1e-3), dict(maxrank=120, abstol=5.0)):
        got, _ = run(pctx, A, **kw)
        assert_same(got, O.OracleLU(A, **kw))


def test_persist_nan(pctx):
    """NaN entries: never selected (Julia's > is false), the certificate treats them as absent."""
    A = rand(1300, 1200, 9)
    A[17, 40] = np.nan
    A[600:610, 500] = np.nan
    kw = dict(maxrank=90)
    got, _ = run(pctx, A, **kw)
    assert_same(got, O.OracleLU(A, **kw))


@pytest.mark.parametrize("epochs", [1, 3])
def test_persist_certificate_fallback(pctx, epochs):
    """Rapidly decaying blocks: the shadow certificate fails part of the way through (uniformly over
    the grid); the persistent launch ends before the pass writes anything, the host resumes at that
    pass with per-pass launches (exact bodies) -- the oracle's bits, and the context keeps the
    persistent form (no give-up)."""
    rng = np.random.default_rng(epochs)
    pctx.check(pctx.lib.tci_set_rrlu_epochs(pctx.h, epochs))
    try:
        for base in (1.05, 1.2, 1.6):
            Q1 = rng.standard_normal((1400, 200))
            Q2 = rng.standard_normal((200, 1300))
            A = (Q1 * base ** -np.arange(200.0)) @ Q2
            for lo in (True, False):
                kw = dict(maxrank=150, reltol=0.0, leftorthogonal=lo)
                got, _ = run(pctx, A, **kw)
                assert_same(got, O.OracleLU(A, **kw))
        assert pctx.lib.tci_rrlu_persist_faulted(pctx.h) == 0
    finally:
        pctx.check(pctx.lib.tci_set_rrlu_epochs(pctx.h, 0))


def test_persist_not_coresident_resumes():
    """Test mode (tci_set_rrlu_persist(ctx, 2)) with two workgroups per CU (TCI_PASS_GRIDX=2): the
    persistent grid is twice what can be resident, its first half waits for the second, gives up
    after 2 ms (ABORT by compare-and-swap on the ticket, st->done = 2) and the factorisation resumes
    with per-pass launches at the pass after the last commit -- the oracle's bits, and the context
    records the give-up."""
    old = os.environ.get("TCI_PASS_GRIDX")
    os.environ["TCI_PASS_GRIDX"] = "2"
    try:
        c = make_ctx(2)
    finally:
        if old is None:
            del os.environ["TCI_PASS_GRIDX"]
        else:
            os.environ["TCI_PASS_GRIDX"] = old
    try:
        A = rand(2100, 1900, 21)
        for lo in (True, False):
            c.check(c.lib.tci_set_rrlu_persist(c.h, 2))  # (resets the give-up flag)
            kw = dict(maxrank=120, leftorthogonal=lo)
            got = T.rrlu(A, ctx=c, **kw)
            assert_same(got, O.OracleLU(A, **kw))
            assert c.lib.tci_rrlu_persist_faulted(c.h) == 1
    finally:
        c.close()
