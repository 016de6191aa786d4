"""Parity at the benchmarked sizes: the rrLU of BASELINE config 2
(4096 x 4096, r = 256) and of the metric matrix (8192 x 8192, r = 256) -- the very seed-0 U[0,1)
matrices bench.py factorises -- bitwise against the CPU oracle (permutations, L, U, npivot,
error), leftorthogonal true and false, with the certified fp16 shadow search on (the default) and
off. Reference: src/matrixlu.jl:346-396 (_optimizerrlu!), benchmark/rrlu.jl:13-18.

The oracle takes ~3 s (4096^2) and ~11 s (8192^2) per factorisation on one core; each oracle
result is computed once per module and shared by the device variants.
"""
import numpy as np
import pytest

import oracle_lib as O

pytestmark = pytest.mark.gpu

T = pytest.importorskip("tci_amd")

_oracle_cache = {}


def oracle(m, n, r, leftorth):
    key = (m, n, r, leftorth)
    if key not in _oracle_cache:
        A = O.fill_uniform(m * n, seed=0).reshape((m, n), order="F")
        _oracle_cache[key] = (A, O.OracleLU(A, maxrank=r, leftorthogonal=leftorth))
    return _oracle_cache[key]


@pytest.fixture(scope="module", params=["shadow", "exact"])
def ctx(request):
    c = T.Context(0)
    c.check(c.lib.tci_set_rrlu_shadow(c.h, int(request.param == "shadow")))
    yield c
    c.close()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("m,n,r", [(4096, 4096, 256), (8192, 8192, 256)])
@pytest.mark.parametrize("leftorth", [True, False])
def test_rrlu_benchmarked_sizes_bitwise(ctx, m, n, r, leftorth):
    A, ref = oracle(m, n, r, leftorth)
    lu = T.rrlu(A, maxrank=r, leftorthogonal=leftorth, ctx=ctx)
    assert lu.npivot == ref.npivot == r
    assert np.array_equal(lu.rowpermutation - 1, ref.rowpermutation)
    assert np.array_equal(lu.colpermutation - 1, ref.colpermutation)
    assert np.array_equal(lu.L, ref.L)
    assert np.array_equal(lu.U, ref.U)
    assert lu.error == ref.error
    assert np.array_equal(T.pivoterrors(lu), ref.pivoterrors)


@pytest.mark.timeout(300)
def test_rrlu_device_inplace_metric_bitwise(ctx):
    """The bench's own entry (tci_rrlu_inplace_d on a device-filled matrix) at the metric size:
    permutations and pivot errors bitwise the oracle's."""
    m = n = 8192
    r = 256
    A, ref = oracle(m, n, r, True)
    W = T.DeviceMatrix(m, n, ctx=ctx)
    W.fill_uniform(seed=0)
    npv, err, rp, cp, pe = T.rrlu_inplace_device(W, maxrank=r)
    W.free()
    assert npv == ref.npivot
    assert np.array_equal(rp[:m] - 1, ref.rowpermutation)
    assert np.array_equal(cp[:n] - 1, ref.colpermutation)
    assert err == ref.error
    assert np.array_equal(pe, ref.pivoterrors)


@pytest.mark.timeout(300)
def test_rrlu_device_copy_metric_bitwise(ctx):
    """bench.py's step as it runs now: rrlu(A) with the copy fused into the initial pass
    (tci_rrlu_copy_d) at the metric size -- permutations, npivot, lu.error and pivot errors bitwise
    the oracle's, and the input untouched."""
    m = n = 8192
    r = 256
    A, ref = oracle(m, n, r, True)
    src = T.DeviceMatrix(m, n, ctx=ctx)
    src.fill_uniform(seed=0)
    W = T.DeviceMatrix(m, n, ctx=ctx)
    npv, err, rp, cp, pe = T.rrlu_inplace_device(W, maxrank=r, src=src)
    untouched = bool(np.array_equal(src.to_host(), A))
    W.free()
    src.free()
    assert untouched
    assert npv == ref.npivot
    assert np.array_equal(rp[:m] - 1, ref.rowpermutation)
    assert np.array_equal(cp[:n] - 1, ref.colpermutation)
    assert err == ref.error
    assert np.array_equal(pe, ref.pivoterrors)
