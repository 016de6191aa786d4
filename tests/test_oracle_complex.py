"""CPU checks of the ComplexF64 rrLU restatement (oracle/tci_oracle.c, orc_rrlu_c128).

Pinned by: the reference's complex argmax known-answer test (test/test_matrixlu.jl:39-52: the
first pivot of rrlu is the abs2 argmax), factorisation identities (A[rowperm, colperm] = L U at
full rank, exact rank revelation) and agreement with the Float64 restatement on real-valued
complex input. Julia's complex division and abs (base/complex.jl) are restated, not executed:
parity at their last ulp is unpinned (Oracle), so those checks carry tolerances.
"""
import cmath
import math

import numpy as np
import pytest

import oracle_lib as O


def julia_argmax(A):
    # first maximum in column-major order (Julia's argmax over a Matrix), 1-based
    flat = np.asarray(A).ravel(order="F")
    i = int(np.argmax(flat))
    return i % A.shape[0] + 1, i // A.shape[0] + 1


def test_complex_first_pivot_is_abs2_argmax(kats):
    k = kats["argmax_complex_3x6"]
    Z = np.array(k["re"], float) + 1j * np.array(k["im"], float)
    lu = O.OracleLUc(Z, maxrank=1)
    assert (lu.rowpermutation[0] + 1, lu.colpermutation[0] + 1) == julia_argmax(np.abs(Z) ** 2)


@pytest.mark.parametrize("shape", [(7, 5), (30, 40), (64, 64)])
@pytest.mark.parametrize("leftorth", [True, False])
def test_complex_full_rank_identity(shape, leftorth):
    rng = np.random.default_rng(sum(shape))
    A = rng.random(shape) + 1j * rng.random(shape) - (0.5 + 0.5j)
    lu = O.OracleLUc(A, leftorthogonal=leftorth)
    assert lu.npivot == min(shape)
    P = A[lu.rowpermutation][:, lu.colpermutation]
    np.testing.assert_allclose(lu.L @ lu.U, P, rtol=0, atol=1e-13)
    d = np.diag(lu.L) if leftorth else np.diag(lu.U[:, : lu.npivot])
    assert np.all(d == 1)
    assert lu.error == 0.0
    # |pivots| descend in magnitude only loosely, but each is the trailing max: never below the
    # next trailing block's entries -- check the first against the global max
    assert lu.pivoterrors[0] == pytest.approx(np.abs(A).max(), rel=1e-15)


def test_complex_rank_revealed():
    rng = np.random.default_rng(5)
    B = (rng.random((40, 3)) + 1j * rng.random((40, 3))) @ (rng.random((3, 50)) - 0.5j)
    lu = O.OracleLUc(B, reltol=1e-12)
    assert lu.npivot == 3
    assert lu.error < 1e-12 * lu.pivoterrors[0]


def test_complex_matches_real_on_real_input():
    rng = np.random.default_rng(6)
    A = rng.random((25, 30))
    for lo in (True, False):
        c = O.OracleLUc(A.astype(complex), leftorthogonal=lo, maxrank=12)
        r = O.OracleLU(A, leftorthogonal=lo, maxrank=12)
        assert c.npivot == r.npivot
        assert np.array_equal(c.rowpermutation, r.rowpermutation)
        assert np.array_equal(c.colpermutation, r.colpermutation)
        np.testing.assert_allclose(c.L.real, r.L, rtol=1e-13, atol=1e-15)
        np.testing.assert_allclose(c.U.real, r.U, rtol=1e-13, atol=1e-15)
        assert np.all(c.L.imag == 0) and np.all(c.U.imag == 0)


def test_complex_nan_raises():
    A = np.ones((4, 4), complex) + np.eye(4)
    A[2, 0] = complex(np.nan, 0)
    with pytest.raises(O.OracleError, match="lu.L contains NaNs"):
        O.OracleLUc(A)


def test_cdiv_and_hypot_restatements():
    rng = np.random.default_rng(7)
    for _ in range(2000):
        e1, e2 = rng.integers(-150, 150, size=2)
        z = complex(*(rng.standard_normal(2) * 2.0 ** e1))
        w = complex(*(rng.standard_normal(2) * 2.0 ** e2))
        q = O.cdiv(z, w)
        ref = z / w
        assert cmath.isclose(q, ref, rel_tol=4e-16), (z, w, q, ref)
        x, y = z.real, z.imag
        assert O.lib().orc_hypot(x, y) == pytest.approx(math.hypot(x, y), rel=2.3e-16)
    assert O.lib().orc_hypot(float("inf"), float("nan")) == float("inf")
    assert math.isnan(O.lib().orc_hypot(1.0, float("nan")))


@pytest.mark.parametrize("leftorth", [True, False])
def test_complex_luci_cross_interpolation(leftorth):
    # MatrixLUCI property (test_matrixluci.jl:6-74): left * right reproduces A exactly on the
    # pivot rows and columns, and A itself at full rank
    rng = np.random.default_rng(8)
    A = rng.random((30, 24)) - 0.5 + 1j * (rng.random((30, 24)) - 0.5)
    ri, ci, pe, left, right = O.luci_c128(A, maxrank=10, leftorthogonal=leftorth)
    assert len(ri) == 10
    approx = left @ right
    np.testing.assert_allclose(approx[ri, :], A[ri, :], rtol=0, atol=1e-13)
    np.testing.assert_allclose(approx[:, ci], A[:, ci], rtol=0, atol=1e-13)
    ri, ci, pe, left, right = O.luci_c128(A, leftorthogonal=leftorth)
    np.testing.assert_allclose(left @ right, A, rtol=0, atol=1e-13)
