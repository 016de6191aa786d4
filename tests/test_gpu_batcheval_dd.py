"""tci_batcheval_dd: batch evaluation from device-resident index tables with the max |Pi| folded into a
device running maximum (the sharded evaluation's per-rank block). Bitwise equal to
tci_batcheval_d (itself checked against the oracle, test_gpu_parity.py) and to the oracle's
batcheval (batcheval.jl:131-175) for integer-exact kinds; the running maximum is updatemaxsample!'s
(tensorci2.jl:636-638) over several batches, NaN-propagating like Julia's max."""
import ctypes as C

import numpy as np
import pytest

import oracle_lib as O

pytestmark = pytest.mark.gpu

T = pytest.importorskip("tci_amd")


@pytest.fixture(scope="module")
def ctx():
    return T.context(0)


def dd(ctx, f, I, J, M, dmax):
    m, nl = I.shape
    n, nr = J.shape
    D = f.localdims[nl] if M else 1
    out = T.DeviceMatrix(m * D, n, ctx=ctx)
    dI = T.DeviceMatrix(I.size // 2 + 1, 1, ctx=ctx)
    dJ = T.DeviceMatrix(J.size // 2 + 1, 1, ctx=ctx)
    try:
        ctx.check(ctx.lib.tci_memcpy_h2d(ctx.h, dI.ptr, T._lib.ptr(I), I.nbytes))
        ctx.check(ctx.lib.tci_memcpy_h2d(ctx.h, dJ.ptr, T._lib.ptr(J), J.nbytes))
        ctx.check(ctx.lib.tci_batcheval_dd(ctx.h, f.h, dI.ptr, m, nl, dJ.ptr, n, nr, M, out.ptr, out.ld, dmax.ptr))
        return out.to_host().copy(order="F")
    finally:
        for x in (out, dI, dJ):
            x.free()


def dmax_value(ctx, dmax):
    bits = np.zeros(1, np.uint64)
    ctx.check(ctx.lib.tci_memcpy_d2h(ctx.h, T._lib.ptr(bits), dmax.ptr, 8))
    return float(bits.view(np.float64)[0])


@pytest.mark.parametrize("M", [0, 1])
def test_dd_equals_d_and_oracle(ctx, M):
    ld = [10] * 8
    f = T.lorentz(ld, ctx=ctx)
    rng = np.random.default_rng(3 + M)
    nl = 3
    I = rng.integers(1, 11, (300, nl)).astype(np.int32)
    J = rng.integers(1, 11, (257, 8 - nl - M)).astype(np.int32)
    dmax = T.DeviceMatrix(2, 1, ctx=ctx)
    try:
        ctx.check(ctx.lib.tci_memcpy_h2d(ctx.h, dmax.ptr, T._lib.ptr(np.zeros(1, np.uint64)), 8))
        got = dd(ctx, f, I, J, M, dmax)
        ref, mx = f.pi(I, J, M)
        assert np.array_equal(got, ref)
        assert dmax_value(ctx, dmax) == mx
        oref, omx = O.batcheval(T.F_LORENTZ, [1.0], ld, I, J, M)
        assert np.array_equal(got, oref.reshape(got.shape, order="F"))
        assert omx == mx
    finally:
        dmax.free()


def test_dd_running_max_and_nan(ctx):
    """The maximum runs over batches (not reset by a call) and propagates NaN like Julia's max."""
    ld = [4] * 6
    T_ = np.random.default_rng(5).random(4 ** 6)
    T_[17] = np.nan
    f = T.table(T_.reshape(ld, order="F"), ctx=ctx)
    rng = np.random.default_rng(7)
    dmax = T.DeviceMatrix(2, 1, ctx=ctx)
    try:
        ctx.check(ctx.lib.tci_memcpy_h2d(ctx.h, dmax.ptr, T._lib.ptr(np.zeros(1, np.uint64)), 8))
        small = [np.array([[1, 1, 1]], np.int32), np.array([[1, 1, 1]], np.int32)]
        dd(ctx, f, small[0], small[1], 0, dmax)
        first = dmax_value(ctx, dmax)
        assert first == abs(T_[0])
        I = rng.integers(1, 5, (40, 3)).astype(np.int32)
        J = rng.integers(1, 5, (30, 3)).astype(np.int32)
        got = dd(ctx, f, I, J, 0, dmax)
        ref, mx = f.pi(I, J, 0)
        assert np.array_equal(got, ref, equal_nan=True)
        assert dmax_value(ctx, dmax) == max(first, mx)
        # the NaN entry (index 18 in 1-based column-major order): (2,1,2,1,1,1)
        dd(ctx, f, np.array([[2, 1, 2]], np.int32), np.array([[1, 1, 1]], np.int32), 0, dmax)
        assert np.isnan(dmax_value(ctx, dmax))
    finally:
        dmax.free()


def test_dd_rejects_host_and_null(ctx):
    f = T.lorentz([3] * 4, ctx=ctx)
    r = ctx.lib.tci_batcheval_dd(ctx.h, f.h, None, 1, 2, None, 1, 2, 0, None, 1, None)
    assert r != 0


@pytest.mark.parametrize("M", [0, 1])
def test_da_equals_d(ctx, M):
    """tci_batcheval_da (host tables, asynchronous upload, device running maximum; the sharded 2-site
    update's evaluation): bitwise tci_batcheval_d's Pi and max, over several back-to-back calls whose
    host tables are overwritten as soon as each call returns."""
    ld = [10] * 8
    f = T.lorentz(ld, ctx=ctx)
    rng = np.random.default_rng(11 + M)
    nl = 4
    dmax = T.DeviceMatrix(2, 1, ctx=ctx)
    outs = [T.DeviceMatrix(200 * (10 if M else 1), 150, ctx=ctx) for _ in range(3)]
    try:
        ctx.check(ctx.lib.tci_memcpy_h2d(ctx.h, dmax.ptr, T._lib.ptr(np.zeros(1, np.uint64)), 8))
        I = np.zeros((200, nl), np.int32)
        J = np.zeros((150, 8 - nl - M), np.int32)
        refs, mxs = [], []
        for out in outs:
            I[:] = rng.integers(1, 11, I.shape)
            J[:] = rng.integers(1, 11, J.shape)
            ctx.check(ctx.lib.tci_batcheval_da(ctx.h, f.h, T._lib.ptr(I), 200, nl, T._lib.ptr(J), 150, J.shape[1], M,
                                               out.ptr, out.ld, dmax.ptr))
            ref, mx = f.pi(I.copy(), J.copy(), M)
            refs.append(ref)
            mxs.append(mx)
        for out, ref in zip(outs, refs):
            assert np.array_equal(out.to_host(), ref)
        assert dmax_value(ctx, dmax) == max(mxs)
    finally:
        dmax.free()
        for o in outs:
            o.free()
