"""Parity at config 5's defining rank, r = 1024, and of the Pi half
of the metric at its benchmarked size.

rrLU at r = 1024, bitwise against the all-core CPU restatement (oracle/cpu_rrlu_omp.c, itself
bitwise equal to the loop-for-loop oracle: tests/test_oracle_kats.py::test_omp_baseline_*):
permutations, L, U, npivot, lu.error and the pivot errors, with the certified fp16 shadow search
on (the default) and off:
  * 16384 x 16384 U[0,1) (the generator of bench.py), leftorthogonal = true;
  * 32768 x 8192 block of config 5's CP-rank-1024 Pi (12 legs of d = 32, the C5 integrand of
    scripts/tci2_configs.py, assembled on the device), leftorthogonal = false -- the 32768-row
    shape and the decaying spectrum of C5 (about 93 write-back epochs over 1024 pivots);
  * 8192 x 8192 with a 2^(-k/3) spectrum over fp64 noise, reltol = 0: the shadow search's exact-
    body fallback (eps >= 2^-7 s |pivot k|) and the per-epoch rescaling through 1024 pivots.
Reference: src/matrixlu.jl:346-396 (_optimizerrlu!), :46-87 (submatrixargmax), :295-322 (addpivot!).

Pi at the metric's size (bench.py extras): 8192 x 8192, L = 20 Lorentzian (integer-exact: bitwise)
and L = 40 quantics oscillatory (exp / sin / pow: device ocml vs glibc, rtol 1e-12), against the
oracle's _batchevaluate_dispatch restatement (batcheval.jl:131-175), maxabs included.
"""
import numpy as np
import pytest

import oracle_lib as O

pytestmark = pytest.mark.gpu

T = pytest.importorskip("tci_amd")

_cpu = {}


def _cp_pi(m, n, seed=2):
    """32768 x 8192 block of the C5 integrand's Pi: f = sum_k prod_t g[k, t, x_t], K = 1024,
    L = 12, d = 32, rows = random 6-leg left sets, columns = random 6-leg right sets."""
    ctx = T.context(0)
    K, L, d = 1024, 12, 32
    g = 0.5 + np.random.default_rng(seed).random((K, L, d))
    f = T.cp_function(g, ctx=ctx)
    rng = np.random.default_rng(seed + 1)
    I = rng.integers(1, d + 1, (m, 6)).astype(np.int32)
    J = rng.integers(1, d + 1, (n, 6)).astype(np.int32)
    Pi, _ = f.pi(I, J, 0)
    f.release()
    return np.asfortranarray(Pi)


def _decaying(m, n, K=1200, seed=5):
    rng = np.random.default_rng(seed)
    U = rng.standard_normal((m, K))
    V = rng.standard_normal((K, n))
    s = 2.0 ** (-np.arange(K) / 3.0)
    A = np.asfortranarray((U * s) @ V)
    A += 1e-17 * rng.standard_normal((m, n))  # below the fp64 floor of the leading values
    return A


def _case(name):
    """(A, CPU result) -- the matrix and the OpenMP oracle's packed factorisation, once per case."""
    if name in _cpu:
        return _cpu[name]
    if name == "uniform16k":
        m = n = 16384
        A = O.fill_uniform(m * n, seed=0).reshape((m, n), order="F")
        kw = dict(maxrank=1024, reltol=1e-14, leftorth=True)
    elif name == "c5_cp":
        m, n = 32768, 8192
        A = _cp_pi(m, n)
        kw = dict(maxrank=1024, reltol=1e-14, leftorth=False)
    else:
        m = n = 8192
        A = _decaying(m, n)
        kw = dict(maxrank=1024, reltol=0.0, leftorth=True)
    w = np.array(A.ravel(order="F"), copy=True)  # ravel of an F-ordered A is a view: never factorise A itself
    npv, err, rp, cp = O.rrlu_inplace_omp(w, m, n, kw["maxrank"], -1, reltol=kw["reltol"], leftorth=kw["leftorth"])
    P = w.reshape((m, n), order="F")
    k = npv
    L = np.tril(P[:, :k])
    U = np.triu(P[:k, :])
    pe = np.concatenate([np.abs(np.diag(P[:k, :k])), [err]])
    if kw["leftorth"]:
        L[np.arange(k), np.arange(k)] = 1.0
    else:
        U[np.arange(k), np.arange(k)] = 1.0
    del w, P
    _cpu[name] = (A, kw, dict(npivot=npv, error=err, rowperm=rp[:m].copy(), colperm=cp[:n].copy(), L=L, U=U, pe=pe))
    return _cpu[name]


@pytest.fixture(scope="module", params=["shadow", "exact"])
def ctx(request):
    c = T.Context(0)
    c.check(c.lib.tci_set_rrlu_shadow(c.h, int(request.param == "shadow")))
    yield c
    c.close()


@pytest.mark.timeout(900)
@pytest.mark.parametrize("case", ["uniform16k", "c5_cp", "decaying8k"])
def test_rrlu_rank1024_bitwise_vs_cpu(ctx, case):
    A, kw, ref = _case(case)
    lu = T.rrlu(A, maxrank=kw["maxrank"], reltol=kw["reltol"], leftorthogonal=kw["leftorth"], ctx=ctx)
    assert lu.npivot == ref["npivot"] and ref["npivot"] > 512
    assert np.array_equal(lu.rowpermutation - 1, ref["rowperm"])
    assert np.array_equal(lu.colpermutation - 1, ref["colperm"])
    assert lu.error == ref["error"]
    assert np.array_equal(T.pivoterrors(lu), ref["pe"])
    assert np.array_equal(lu.L, ref["L"])
    assert np.array_equal(lu.U, ref["U"])


@pytest.mark.timeout(600)
def test_pi_lorentz_metric_size_bitwise():
    """bench.py's pi_lorentz: 8192 x 8192, L = 20, d = 10, seed-1 index tables."""
    ctx = T.context(0)
    rng = np.random.default_rng(1)
    m = n = 8192
    I = rng.integers(1, 11, (m, 10)).astype(np.int32)
    J = rng.integers(1, 11, (n, 10)).astype(np.int32)
    f = T.lorentz([10] * 20, ctx=ctx)
    got, gmx = f.pi(I, J, 0)
    ref, rmx = O.batcheval(1, [1.0], [10] * 20, I, J, 0)
    assert np.array_equal(got, ref[:, 0, :])
    assert gmx == rmx


@pytest.mark.timeout(600)
def test_pi_quantics_metric_size():
    """bench.py's pi_quantics_osc: 8192 x 8192 of the 40-bit quantics oscillatory integrand
    (test_tensorci2.jl:437), rtol 1e-12 (transcendentals: ocml vs glibc)."""
    ctx = T.context(0)
    rng = np.random.default_rng(1)
    m = n = 8192
    rng.integers(1, 11, (m, 10))
    rng.integers(1, 11, (n, 10))  # the bench draws the Lorentz tables first from the same stream
    Ib = rng.integers(1, 3, (m, 20)).astype(np.int32)
    Jb = rng.integers(1, 3, (n, 20)).astype(np.int32)
    f = T.GPUBatchEvaluator(5, T.batcheval.QOSC_PARAMS, [2] * 40, ctx=ctx)
    got, gmx = f.pi(Ib, Jb, 0)
    ref, rmx = O.batcheval(5, T.batcheval.QOSC_PARAMS, [2] * 40, Ib, Jb, 0)
    ref = ref[:, 0, :]
    np.testing.assert_allclose(got, ref, rtol=1e-12, atol=1e-13 * np.abs(ref).max())
    assert gmx == pytest.approx(rmx, rel=1e-12)
