"""The device-resident sweep (tci_sweep_small.hip: whole sweep2site! iterations in one launch while
every bond's Pi fits the one-workgroup rrLU) against the per-bond native loop (tci_sweep.cpp,
one tci_update_pivots_h per bond) and the oracle: identical ranks, pivot sets, history, bond and
pivot errors and maxsamplevalue, bit for bit, for every staged catalog kind, both sweep
strategies and strict nesting, a run whose bonds outgrow the small path part of the way through
an iteration (the host loop resumes at the kernel's resume point), the NaN error of the rrLU and
fillsitetensors!'s maxsample update (tci_tci2_fill_maxsample).
Reference: tensorci2.jl:1195-1258 (sweep2site!), :512-529 (kronecker), :1214-1216 (union),
:281-289 (updateerrors!), :636-638 (updatemaxsample!), globalsearch.jl:202-208
(fillsitetensors!), matrixlu.jl:376-381 (the NaN checks).
"""
import ctypes as C

import numpy as np
import pytest

import oracle_lib as O

pytestmark = pytest.mark.gpu

T = pytest.importorskip("tci_amd")
import tci_amd.tensorci2 as TT  # noqa: E402


def _table(ld, seed):
    rng = np.random.default_rng(seed)
    A = rng.random(ld)
    return A


CASES = {
    "sum": (lambda c: T.sum_([4] * 6, ctx=c), [4] * 6, dict(tolerance=1e-12)),
    "lorentz": (lambda c: T.lorentz([10] * 8, ctx=c), [10] * 8, dict(tolerance=1e-8)),
    "lorentz_fwd": (lambda c: T.lorentz([6] * 7, ctx=c), [6] * 7, dict(tolerance=1e-10, sweepstrategy="forward")),
    "lorentz_bwd": (lambda c: T.lorentz([6] * 7, ctx=c), [6] * 7, dict(tolerance=1e-10, sweepstrategy="backward")),
    "lorentz_strict": (lambda c: T.lorentz([6] * 6, ctx=c), [6] * 6, dict(tolerance=1e-10, strictlynested=True)),
    "lorentz_maxbond": (lambda c: T.lorentz([10] * 6, ctx=c), [10] * 6, dict(tolerance=1e-14, maxbonddim=7, maxiter=5)),
    "table": (lambda c: T.table(_table([3, 4, 3, 5, 2], 3), ctx=c), [3, 4, 3, 5, 2], dict(tolerance=1e-12)),
    "gauss20": (lambda c: T.gauss([16] * 20, 0.05, 8.5, ctx=c), [16] * 20, dict(tolerance=1e-10, maxbonddim=512)),
    "qosc40": (lambda c: T.quantics_osc(40, ctx=c), [2] * 40, dict(tolerance=1e-8)),
    "qexp30": (lambda c: T.quantics_exp(30, 1.0, 3.0, 0.5, 0.7, ctx=c), [2] * 30, dict(tolerance=1e-12)),
    # bonds outgrow (m|1) n <= 16384 part of the way: the host loop takes over mid-iteration
    "lorentz_resume": (lambda c: T.lorentz([12] * 7, ctx=c), [12] * 7, dict(tolerance=1e-15, maxiter=4)),
}


def _run(f, ld, small, **kw):
    ctx = f.ctx
    ctx.check(ctx.lib.tci_set_sweep_small(ctx.h, int(small)))
    try:
        return T.crossinterpolate2(f, ld, [T.optfirstpivot(f, ld)], nsearchglobalpivot=0, **kw)
    finally:
        ctx.check(ctx.lib.tci_set_sweep_small(ctx.h, 1))


def _same(t1, t2):
    L = len(t1.localdims)
    assert t1.maxsamplevalue == t2.maxsamplevalue
    assert np.array_equal(t1.bonderrors, t2.bonderrors)
    assert np.array_equal(t1.pivoterrors, t2.pivoterrors)
    for b in range(L):
        assert np.array_equal(t1.Iset[b], t2.Iset[b]), b
        assert np.array_equal(t1.Jset[b], t2.Jset[b]), b
        assert np.array_equal(t1.sitetensors[b], t2.sitetensors[b]), b
    for h1, h2 in zip(t1.Iset_history[-1], t2.Iset_history[-1]):
        assert np.array_equal(h1, h2)
    for h1, h2 in zip(t1.Jset_history[-1], t2.Jset_history[-1]):
        assert np.array_equal(h1, h2)


@pytest.mark.parametrize("name", list(CASES))
def test_device_sweep_equals_per_bond_loop(name):
    ctx = T.context(0)
    mk, ld, kw = CASES[name]
    f = mk(ctx)
    t1, r1, e1 = _run(f, ld, True, **kw)
    t2, r2, e2 = _run(f, ld, False, **kw)
    assert r1 == r2 and list(e1) == list(e2)
    _same(t1, t2)
    if name == "lorentz_resume":
        assert max(r1) * 12 > 128  # some bond's Pi ((r d) x (r d)) left the small path


@pytest.mark.parametrize("name", ["lorentz", "qosc40", "gauss20", "lorentz_fwd"])
def test_device_sweep_vs_oracle(name):
    ctx = T.context(0)
    mk, ld, kw = CASES[name]
    f = mk(ctx)
    p0 = T.optfirstpivot(f, ld)
    tci, ranks, errors = T.crossinterpolate2(f, ld, [p0], nsearchglobalpivot=0, **kw)
    okw = {k: v for k, v in kw.items() if k in ("tolerance", "maxbonddim", "maxiter", "sweepstrategy")}
    rt, rranks, rerrors = O.crossinterpolate2(f.kind, f.params, ld, [p0], **okw)
    assert list(ranks) == list(rranks)
    if f.kind in (T.batcheval.F_SUM, T.batcheval.F_LORENTZ, T.batcheval.F_TABLE):
        assert list(errors) == list(rerrors)  # integer-exact integrands: bitwise, pivots included
        for p in range(len(ld)):
            assert np.array_equal(tci.Iset[p], rt.Iset(p)), p
            assert np.array_equal(tci.Jset[p], rt.Jset(p)), p
    else:
        # exp / sin / pow: ocml vs glibc ulps move near-tied pivots (test_config_golden.py's bar)
        np.testing.assert_allclose(errors, rerrors, rtol=0, atol=1e-10)


def test_device_sweep_nan_error_matches():
    """A NaN in Pi: both paths raise the rrLU's "lu.L/U contains NaNs" with the same message."""
    ctx = T.context(0)
    ld = [3, 3, 3, 3]
    A = _table(ld, 5)
    A[1, 0, 0, 0] = np.nan
    f = T.table(A, ctx=ctx)
    msgs = []
    for small in (True, False):
        ctx.check(ctx.lib.tci_set_sweep_small(ctx.h, int(small)))
        try:
            with pytest.raises(T.TCIError) as ei:
                T.crossinterpolate2(f, ld, [[1, 1, 1, 1]], tolerance=1e-12, nsearchglobalpivot=0)
            msgs.append(str(ei.value))
        finally:
            ctx.check(ctx.lib.tci_set_sweep_small(ctx.h, 1))
    assert msgs[0] == msgs[1] and "NaN" in msgs[0]


def test_fill_maxsample_native_equals_loop():
    """tci_tci2_fill_maxsample == fillsitetensors!(solve=false)'s per-site max |Pi1| loop."""
    ctx = T.context(0)
    ld = [2] * 24
    f = T.quantics_osc(24, ctx=ctx)
    tci, _, _ = T.crossinterpolate2(f, ld, [T.optfirstpivot(f, ld)], tolerance=1e-8, nsearchglobalpivot=0,
                                    maxiter=2)
    tci.maxsamplevalue = 0.0
    h = tci._native_h
    lib = ctx.lib
    # push the current state, run the native fill, compare with the Python loop
    tci._sweep2site_native(f, 0, 1, 1e-8, TT.INT64_MAX, "backandforth", False, fill="max")
    native = tci.maxsamplevalue
    tci.maxsamplevalue = 0.0
    tci.fillsitetensors(f, solve=False)
    assert native == tci.maxsamplevalue and native > 0.0
    assert h is not None and lib is not None


@pytest.mark.parametrize("name", ["lorentz", "qosc40", "table", "gauss20", "qexp30", "sum"])
def test_fill_solve_native_equals_oracle_solve(name):
    """fillsitetensors! with the solves (globalsearch.jl:202-208, setsitetensor! tensorci2.jl:599-629)
    in one device launch (tci_tci2_fill_solve): maxsamplevalue bitwise the per-site loop's; every
    site tensor T = Pi1 P^-1 bitwise the oracle's getrf / getrs restatement (orc_sitetensor_solve) on
    the same Pi1 and P (the kernel keeps its operation order), and within rtol 1e-10 of the host
    loop's device solve (tci_sitetensor_h, K5: blocked, its own summation order)."""
    ctx = T.context(0)
    mk, ld, kw = CASES[name]
    f = mk(ctx)
    kw = dict(kw, maxiter=2)
    kw.pop("sweepstrategy", None)
    tci, _, _ = T.crossinterpolate2(f, ld, [T.optfirstpivot(f, ld)], nsearchglobalpivot=0, **kw)
    tci.maxsamplevalue = 0.0
    assert tci._sweep2site_native(f, 0, 1, 1e-8, TT.INT64_MAX, "backandforth", False, fill="solve")
    native_ms = tci.maxsamplevalue
    native_T = [t.copy() for t in tci.sitetensors]
    tci.maxsamplevalue = 0.0
    tci.fillsitetensors(f, solve=True)  # the host loop (tci_sitetensor_h per site)
    assert native_ms == tci.maxsamplevalue and native_ms > 0.0
    L = len(ld)
    for p in range(L):
        Ib, Jb = tci.Iset[p], tci.Jset[p]
        Pi1 = f.pi(Ib, Jb, 1)[0].reshape((len(Ib) * ld[p], len(Jb)), order="F")
        if p < L - 1:
            P = f.pi(tci.Iset[p + 1], Jb, 0)[0]
            ref = O.sitetensor_solve(P, Pi1)
        else:
            ref = Pi1
        got = native_T[p].reshape(ref.shape, order="F")
        assert np.array_equal(got, ref), (name, p)
        host = tci.sitetensors[p].reshape(ref.shape, order="F")
        assert np.allclose(got, host, rtol=1e-10, atol=1e-12 * native_ms), (name, p)


@pytest.mark.parametrize("lazy", [False, True])
def test_sweep2site_fill_solve_in_launch(lazy):
    """crossinterpolate2 with the reference's work (fillsitetensors! solving every site tensor after
    each sweep2site!, lazy=False: tci_tci2_sweep2site_fillsolve) and with the solves skipped
    (lazy=True): identical ranks, errors, sets and final tensors; the device path equals the host
    loop (tci_set_sweep_small 0) on ranks / errors / sets bit for bit."""
    ctx = T.context(0)
    ld = [2] * 30
    f = T.quantics_osc(30, ctx=ctx)
    p0 = [T.optfirstpivot(f, ld)]
    out = []
    for small in (1, 0):
        ctx.check(ctx.lib.tci_set_sweep_small(ctx.h, small))
        try:
            out.append(T.crossinterpolate2(f, ld, p0, tolerance=1e-8, nsearchglobalpivot=0, lazy_sitetensors=lazy))
        finally:
            ctx.check(ctx.lib.tci_set_sweep_small(ctx.h, 1))
    (t1, r1, e1), (t2, r2, e2) = out
    assert r1 == r2 and list(e1) == list(e2)
    _same(t1, t2)


def test_bulk_set_transfer_roundtrip():
    ctx = T.context(0)
    L = 5
    lib = ctx.lib
    h = C.c_void_p()
    ctx.check(lib.tci_tci2_create(ctx.h, L, np.array([3] * L, np.int32), C.byref(h)))
    try:
        rng = np.random.default_rng(0)
        sets = [rng.integers(1, 4, (int(c), p)).astype(np.int32) for p, c in enumerate([1, 4, 7, 2, 5])]
        counts = np.array([len(s) for s in sets], np.int64)
        packed = np.concatenate([s.ravel() for s in sets]).astype(np.int32)
        ctx.check(lib.tci_tci2_set_sets(h, 0, counts.ctypes.data_as(C.c_void_p), packed.ctypes.data_as(C.c_void_p)))
        got_counts = np.zeros(L, np.int64)
        ctx.check(lib.tci_tci2_get_sets(h, 0, got_counts.ctypes.data_as(C.c_void_p), None, 0))
        assert np.array_equal(got_counts, counts)
        out = np.zeros(len(packed), np.int32)
        ctx.check(lib.tci_tci2_get_sets(h, 0, got_counts.ctypes.data_as(C.c_void_p), out.ctypes.data_as(C.c_void_p),
                                        len(out)))
        assert np.array_equal(out, packed)
        # per-set getter agrees
        for p in range(1, L):
            cnt = C.c_int64()
            a = np.zeros((int(counts[p]), p), np.int32)
            ctx.check(lib.tci_tci2_get_set(h, 0, p, a.ctypes.data_as(C.c_void_p), counts[p], C.byref(cnt)))
            assert np.array_equal(a, sets[p])
        with pytest.raises(T.TCIArgumentError):  # capacity too small
            ctx.check(lib.tci_tci2_get_sets(h, 0, got_counts.ctypes.data_as(C.c_void_p),
                                            out.ctypes.data_as(C.c_void_p), 3))
    finally:
        lib.tci_tci2_destroy(h)


@pytest.mark.parametrize("name", ["lorentz", "qosc40", "table", "lorentz_maxbond"])
@pytest.mark.parametrize("direction,tensors", [("forward", True), ("backward", True), ("backward", False)])
def test_device_sweep1site_equals_host_loop(name, direction, tensors):
    """sweep1site! (tensorci2.jl:659-725) in one launch (tci_tci2_sweep1site) against the host loop
    (one tci_update_pivots_h per bond): sets, bond / pivot errors, maxsamplevalue and the site
    tensors (MatrixLUCI left / right factors and the last site's Pi1) bit for bit, with the
    history untouched."""
    ctx = T.context(0)
    mk, ld, kw = CASES[name]
    f = mk(ctx)
    kw = dict(kw, maxiter=2)
    kw.pop("sweepstrategy", None)
    base, _, _ = T.crossinterpolate2(f, ld, [T.optfirstpivot(f, ld)], nsearchglobalpivot=0, **kw)
    out = []
    for small in (True, False):
        t = TT.TensorCI2.from_sets(f, ld, [s.copy() for s in base.Iset], [s.copy() for s in base.Jset])
        t.Iset_history = [[s.copy() for s in base.Iset_history[-1]]]
        t.Jset_history = [[s.copy() for s in base.Jset_history[-1]]]
        t.maxsamplevalue = base.maxsamplevalue
        t.bonderrors = base.bonderrors.copy()
        ctx.check(ctx.lib.tci_set_sweep_small(ctx.h, int(small)))
        try:
            t.sweep1site(f, direction, abstol=1e-9 * base.maxsamplevalue, maxbonddim=kw.get("maxbonddim", TT.INT64_MAX),
                         updatetensors=tensors)
        finally:
            ctx.check(ctx.lib.tci_set_sweep_small(ctx.h, 1))
        out.append(t)
    _same(out[0], out[1])
    assert all(np.array_equal(a, b) for a, b in zip(out[0].Iset_history[-1], base.Iset_history[-1]))
