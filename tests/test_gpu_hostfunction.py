"""The user's own f on the device rrLU path (VERDICT r2 missing #1): a plain Python
callable / vectorized function / user BatchEvaluator wrapped by HostFunctionEvaluator is
evaluated on the host through the tci_func_create_host callback, and crossinterpolate2 runs the
rest -- maxabs, rrLU, factors, site-tensor solves, the native sweep driver -- on the GPU.

Reference: the generic dispatch batcheval.jl:131-175 (f called per point), the BatchEvaluator
route :196-214 and ThreadedBatchEvaluator :247-308 (threaded == serial, test_batcheval.jl:48-84).
The Lorentzian written as Python, 1.0 / (sum(v*v) + 1.0), is integer-exact like the oracle's
catalog kind, so ranks, index sets, pivot errors and maxsamplevalue are compared bitwise.
"""
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


def lorentz_point(x):
    return 1.0 / (sum(v * v for v in x) + 1.0)


def lorentz_vec(X):
    X = np.asarray(X, np.int64)
    return 1.0 / ((X * X).sum(axis=1).astype(np.float64) + 1.0)


class LorentzBatch:
    """A user BatchEvaluator: (f)(Iset, Jset, Val(M)) -> (|I|, d..., |J|) array."""

    def __init__(self, localdims):
        self.localdims = localdims

    def __call__(self, I, J, M):
        m, nl = I.shape
        n = J.shape[0]
        sI = (I.astype(np.int64) ** 2).sum(1)
        sJ = (J.astype(np.int64) ** 2).sum(1)
        if M == 0:
            s = sI[:, None] + sJ[None, :]
            return 1.0 / (s.astype(np.float64) + 1.0)
        d = self.localdims[nl]
        c = np.arange(1, d + 1, dtype=np.int64) ** 2
        s = sI[:, None, None] + c[None, :, None] + sJ[None, None, :]
        return 1.0 / (s.astype(np.float64) + 1.0)


def _compare(tci, ranks, errors, rt, rranks, rerrors):
    assert ranks == rranks
    assert errors == rerrors  # bitwise: integer-exact f, identical rrLU arithmetic
    for p in range(len(tci.localdims)):
        assert np.array_equal(tci.Iset[p], rt.Iset(p)), p
        assert np.array_equal(tci.Jset[p], rt.Jset(p)), p
    assert np.array_equal(tci.pivoterrors, rt.pivoterrors)
    assert tci.maxsamplevalue == rt.maxsamplevalue
    for p in range(len(tci.localdims)):
        ref = rt.sitetensor(p)
        np.testing.assert_allclose(tci.sitetensors[p], ref, rtol=1e-9, atol=1e-12 * max(1.0, np.abs(ref).max()))


@pytest.mark.parametrize("mode", ["pointwise", "threads", "vectorized", "batch"])
def test_host_function_tci2_bitwise_vs_oracle(ctx, mode):
    ld = [10] * 6
    kw = dict(tolerance=1e-10, maxiter=10)
    if mode == "pointwise":
        f = T.HostFunctionEvaluator(lorentz_point, ld, ctx=ctx)
    elif mode == "threads":
        f = T.HostFunctionEvaluator(lorentz_point, ld, ctx=ctx, threads=4)
    elif mode == "vectorized":
        f = T.HostFunctionEvaluator(lorentz_vec, ld, ctx=ctx, vectorized=True)
    else:
        f = T.HostFunctionEvaluator(LorentzBatch(ld), ld, ctx=ctx, batch=True)
    tci, ranks, errors = T.crossinterpolate2(f, nsearchglobalpivot=0, **kw)
    rt, rranks, rerrors = O.crossinterpolate2(1, [1.0], ld, **kw)
    _compare(tci, ranks, errors, rt, rranks, rerrors)
    assert f.nbatches > 0 and f.npoints > 0
    # the sweeps went through the native driver (one ABI call per sweep, Pi from the callback)
    assert getattr(tci, "_native_h", None) is not None


def test_host_function_config1_and_timing_line(ctx):
    """BASELINE config 1 (README 8d Lorentzian, d = 10, tol 1e-8) with f a plain Python function,
    against the oracle; prints the host / total time split."""
    import time
    ld = [10] * 8
    f = T.HostFunctionEvaluator(lorentz_vec, ld, ctx=ctx, vectorized=True)
    t0 = time.perf_counter()
    tci, ranks, errors = T.crossinterpolate2(f, tolerance=1e-8, nsearchglobalpivot=0)
    wall = time.perf_counter() - t0
    rt, rranks, rerrors = O.crossinterpolate2(1, [1.0], ld, tolerance=1e-8)
    _compare(tci, ranks, errors, rt, rranks, rerrors)
    print(f"\nhost-function C1: wall {wall * 1e3:.1f} ms, host f {f.host_seconds * 1e3:.1f} ms over "
          f"{f.nbatches} batches / {f.npoints} points, ranks {ranks}")


def test_host_function_default_global_search(ctx):
    """With the default (random) global pivot search the scalar calls f(x) and the device batches
    both come from the same host f; the result must interpolate f."""
    ld = [10] * 5
    f = T.HostFunctionEvaluator(lorentz_point, ld, ctx=ctx)
    tci, ranks, errors = T.crossinterpolate2(f, tolerance=1e-10, maxiter=8)
    rng = np.random.default_rng(3)
    X = np.stack([rng.integers(1, 11, 200) for _ in ld], axis=1)
    got = tci.evaluate_many(X, ctx=ctx)
    ref = np.array([lorentz_point(list(x)) for x in X])
    np.testing.assert_allclose(got, ref, rtol=0, atol=1e-8)


def test_host_function_equals_device_catalog(ctx):
    """Pi of the host Lorentzian == Pi of the device catalog kind, bitwise (2-site update and
    site tensors through the same entries)."""
    ld = [7] * 4
    fh = T.HostFunctionEvaluator(lorentz_vec, ld, ctx=ctx, vectorized=True)
    fd = T.lorentz(ld, ctx=ctx)
    rng = np.random.default_rng(1)
    I = rng.integers(1, 8, (37, 2)).astype(np.int32)
    for M in (0, 1):
        J = rng.integers(1, 8, (29, 2 - M)).astype(np.int32)
        a, ma = fh.pi(I, J, M)
        b, mb = fd.pi(I, J, M)
        assert np.array_equal(a, b) and ma == mb
        # through the device entry (callback -> HBM -> maxabs kernel -> host)
        import ctypes as C
        D = ld[2] if M else 1
        out = np.zeros(37 * D * 29)
        mx = C.c_double()
        ctx.check(ctx.lib.tci_batcheval_h(ctx.h, fh.h, T._lib.ptr(I), 37, 2, T._lib.ptr(J), 29, 2 - M, M,
                                          T._lib.ptr(out), 37 * D, C.byref(mx)))
        assert np.array_equal(out.reshape((37 * D, 29), order="F"), b) and mx.value == mb


def test_host_function_nan_maxsample_and_error_propagation(ctx):
    ld = [4] * 4

    calls = [0]

    def bad(x):  # fails inside the first sweep's batches
        calls[0] += 1
        if calls[0] == 30:
            raise KeyError("boom")
        return float(sum(x))

    f = T.HostFunctionEvaluator(bad, ld, ctx=ctx)
    with pytest.raises(KeyError):
        T.crossinterpolate2(f, tolerance=1e-10, maxiter=3, nsearchglobalpivot=0)
    with pytest.raises(ValueError):  # widths that do not add up to L
        f.pi(np.ones((2, 2), np.int32), np.ones((3, 1), np.int32), 0)
    # the context stays usable after the failed call
    g = T.HostFunctionEvaluator(lambda x: float(sum(x)), ld, ctx=ctx)
    tci, ranks, errors = T.crossinterpolate2(g, tolerance=1e-10, maxiter=3, nsearchglobalpivot=0)
    rt, rranks, rerrors = O.crossinterpolate2(0, [0.0], ld, tolerance=1e-10, maxiter=3)
    assert ranks == rranks
    # NaN propagates into maxsamplevalue like Julia's max (util.jl:34-43)
    h = T.HostFunctionEvaluator(lambda x: float("nan") if x == [1, 1, 1, 2] else 1.0, ld, ctx=ctx)
    _, mx = h.pi(np.ones((1, 3), np.int32), np.array([[1], [2]], np.int32), 0)
    assert np.isnan(mx)
    import ctypes as C
    out = np.zeros(2)
    m = C.c_double()
    ctx.check(ctx.lib.tci_batcheval_h(ctx.h, h.h, T._lib.ptr(np.ones((1, 3), np.int32)), 1, 3,
                                      T._lib.ptr(np.array([[1], [2]], np.int32)), 2, 1, 0, T._lib.ptr(out), 1,
                                      C.byref(m)))
    assert np.isnan(m.value)


def test_host_function_device_memo(ctx):
    """CachedFunction over a host f keeps its memo in HBM: only distinct misses reach the host."""
    ld = [6] * 5
    calls = []

    def f(X):
        calls.append(len(X))
        return lorentz_vec(X)

    fh = T.HostFunctionEvaluator(f, ld, ctx=ctx, vectorized=True)
    cf = T.CachedFunction(fh, ld)
    assert cf._memo is not None
    rng = np.random.default_rng(2)
    I = rng.integers(1, 7, (50, 2)).astype(np.int32)
    J = rng.integers(1, 7, (40, 3)).astype(np.int32)
    a, _ = cf.pi(I, J, 0)
    npts = sum(calls)
    distinct = len({tuple(i) + tuple(j) for i in I.tolist() for j in J.tolist()})
    assert npts == distinct
    b, _ = cf.pi(I, J, 0)  # all hits: no host call
    assert sum(calls) == npts
    assert np.array_equal(a, b) and np.array_equal(a, T.lorentz(ld, ctx=ctx).pi(I, J, 0)[0])


def test_host_function_complex_scaled(ctx):
    """ComplexScaledEvaluator over a host f: the complex Lorentzian of test_tensorci2.jl:246-249
    with the real part from Python, equal to the device catalog version."""
    ld = [10] * 5
    coeff = 0.5 - 1.5j
    fh = T.ComplexScaledEvaluator(coeff, T.HostFunctionEvaluator(lorentz_vec, ld, ctx=ctx, vectorized=True))
    fd = T.ComplexScaledEvaluator(coeff, T.lorentz(ld, ctx=ctx))
    kw = dict(tolerance=1e-10, maxiter=6, nsearchglobalpivot=0)
    t1, r1, e1 = T.crossinterpolate2(fh, **kw)
    t2, r2, e2 = T.crossinterpolate2(fd, **kw)
    assert r1 == r2 and e1 == e2
    for p in range(len(ld)):
        assert np.array_equal(t1.Iset[p], t2.Iset[p])


def test_checkbatchevaluatable_accepts_every_host_evaluator(ctx):
    """checkbatchevaluatable=true accepts any BatchEvaluator (tensorci2.jl:1044): the pointwise and
    threaded HostFunctionEvaluator forms expose the batch interface too."""
    ld = [6] * 4
    ref = None
    for kw in ({}, {"threads": 2}, {"vectorized": True}):
        fn = lorentz_vec if kw.get("vectorized") else lorentz_point
        f = T.HostFunctionEvaluator(fn, ld, ctx=ctx, **kw)
        tci, ranks, errors = T.crossinterpolate2(f, tolerance=1e-10, maxiter=4, nsearchglobalpivot=0,
                                                 checkbatchevaluatable=True)
        ref = ref or (ranks, errors)
        assert (ranks, errors) == ref


def test_failed_native_sweep_leaves_mirror_on_native_state(ctx):
    """when a native sweep fails part-way (here the host f raises in the second
    iteration), the Python mirror must show the native object's half-updated sets -- as the
    reference's TensorCI2 is left half-updated when a sweep throws -- not the stale copy."""
    ld = [5] * 5
    calls = [0]

    def f(X):
        calls[0] += 1
        if calls[0] == 16:  # 1 (initial pivot) + 8 bonds + 5 Pi1 in iteration 1; then mid-sweep
            raise KeyError("boom")
        return lorentz_vec(X)

    fh = T.HostFunctionEvaluator(f, ld, ctx=ctx, vectorized=True)
    tci = T.TensorCI2.from_function(fh, ld, None)
    with pytest.raises(KeyError):
        tci.optimize(fh, tolerance=1e-12, maxiter=4, nsearchglobalpivot=0)
    assert getattr(tci, "_native_h", None) is not None
    native = [tci._native_counts(0)[p] for p in range(len(ld))]
    assert [len(s) for s in tci.Iset] == native
