"""rrlu(A) with the copy fused into the first pass (tci_rrlu_copy_d, matrixlu.jl:455-463:
`rrlu!(copy(A))`): the input stays untouched, and the permutations, npivot, lu.error, the pivot
errors and the work matrix's final (stale) contents are bitwise those of an explicit copy followed
by tci_rrlu_inplace_d -- on the pass pipeline (the copy fused into the initial argmax pass: odd
shapes, a different leading dimension for the input, both orientations, the two-level epoch) and on
the one-launch small / mid paths (an explicit copy first). The metric configuration through the
fused copy is checked against the oracle in tests/test_gpu_benchsizes.py."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

T = pytest.importorskip("tci_amd")


@pytest.fixture(scope="module")
def ctx():
    c = T.Context(0)
    yield c
    c.close()


def _host(dm):
    return dm.to_host().copy(order="F")


def _run(ctx, m, n, r, ld_src=None, leftorth=True, seed=3, epochs=0):
    ctx.check(ctx.lib.tci_set_rrlu_epochs(ctx.h, epochs))
    try:
        A = T.DeviceMatrix(m, n, ctx=ctx, ld=ld_src)
        A.fill_uniform(seed=seed)
        before = _host(A)
        W1 = T.DeviceMatrix(m, n, ctx=ctx)
        W2 = T.DeviceMatrix(m, n, ctx=ctx)
        # reference: explicit copy (through the host: the two leading dimensions differ), in place
        W1.upload(before)
        ref = T.rrlu_inplace_device(W1, maxrank=r, leftorthogonal=leftorth)
        got = T.rrlu_inplace_device(W2, maxrank=r, leftorthogonal=leftorth, src=A)
        res = {"npivot": got[0] == ref[0], "error": got[1] == ref[1] or (np.isnan(got[1]) and np.isnan(ref[1])),
               "rowperm": bool(np.array_equal(got[2], ref[2])), "colperm": bool(np.array_equal(got[3], ref[3])),
               "pivoterrors": bool(np.array_equal(got[4], ref[4])),
               "work_matrix": bool(np.array_equal(_host(W2), _host(W1))),
               "input_untouched": bool(np.array_equal(_host(A), before))}
        for x in (A, W1, W2):
            x.free()
        return res, got, before
    finally:
        ctx.check(ctx.lib.tci_set_rrlu_epochs(ctx.h, 0))


@pytest.mark.parametrize("m,n,r,ld_src,leftorth,epochs", [
    (3001, 2501, 200, 3008, True, 0),    # pass pipeline, odd shape, input ld != work ld
    (3001, 2501, 200, 3001, True, 0),    # odd input ld (== m): copied first, not read as row pairs
    (1999, 1800, 100, 2003, False, 0),   # odd input ld > m
    (2500, 3100, 150, None, False, 0),   # right-orthogonal
    (4100, 4000, 120, 4112, True, 3),    # two-level epoch forced (refresh, EXT, deep write-back)
    (90, 70, 70, 96, True, 0),           # one-workgroup small path (explicit copy first)
    (700, 640, 300, None, True, 0),      # mid-size / pass pipeline
])
def test_rrlu_copy_equals_copy_then_inplace(ctx, m, n, r, ld_src, leftorth, epochs):
    res, _, _ = _run(ctx, m, n, r, ld_src, leftorth, epochs=epochs)
    assert all(res.values()), res


def test_rrlu_copy_rejects_overlap(ctx):
    A = T.DeviceMatrix(64, 64, ctx=ctx)
    import ctypes as C
    npv, err = C.c_int64(), C.c_double()
    try:
        st = ctx.lib.tci_rrlu_copy_d(ctx.h, A.ptr, A.ld, A.ptr, 64, 64, A.ld, 10, 1e-14, 0.0, 1, None, None,
                                     C.byref(npv), C.byref(err), None)
        assert st != 0
    finally:
        A.free()
