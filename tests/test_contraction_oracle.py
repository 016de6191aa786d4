"""CPU tests of the contraction path's oracle and host logic (contraction.jl).

Pinned by the reference's own properties (test/test_contraction.jl): the contraction of two MPOs
evaluates to the product of their matrices (`_tomat(ab) ≈ _tomat(a) * _tomat(b)`, :94), also for
an MPO times an MPS (:175-176), on the reference's test shapes (N = 4, bonds [1,2,3,2,1], local
dims 2 x 3 x 2). The reference draws complex random cores; the Float64 tests use real ones, the
ComplexF64 ones at the end complex ones.
"""
import itertools

import numpy as np
import pytest

import oracle_lib as O

T = pytest.importorskip("tci_amd")
from tci_amd.contraction import (_as_mpo_right, _contractsitetensors, _mpo_params, contract_naive, tomat,  # noqa: E402
                                 tovec)

F_MPO = 9


def gen_tto_tto(seed=0, N=4, bonds=(1, 2, 3, 2, 1), d1=2, d2=3, d3=2):
    rng = np.random.default_rng(seed)
    A = [rng.random((bonds[n], d1, d2, bonds[n + 1])) for n in range(N)]
    B = [rng.random((bonds[n], d2, d3, bonds[n + 1])) for n in range(N)]
    return A, B


def fused_index_value(ref, x, d1s, d3s):
    """(A * B)[x] for fused indices x_n = s1 + d1 (s3 - 1) (contraction.jl:226-237)."""
    i = j = 0
    si = sj = 1
    for n, xn in enumerate(x):
        s1, s3 = (xn - 1) % d1s[n], (xn - 1) // d1s[n]
        i += s1 * si
        j += s3 * sj
        si *= d1s[n]
        sj *= d3s[n]
    return ref[i, j]


def test_oracle_mpo_matches_matrix_product():
    A, B = gen_tto_tto()
    ref = tomat(A) @ tomat(B)
    p = _mpo_params(A, B)
    ld = [4] * 4
    err = 0.0
    for x in itertools.product(*[range(1, 5)] * 4):
        err = max(err, abs(O.feval(F_MPO, p, ld, list(x)) - fused_index_value(ref, x, [2] * 4, [2] * 4)))
    assert err <= 1e-12 * np.abs(ref).max()


@pytest.mark.parametrize("N", [1, 2, 5])
def test_oracle_mpo_lengths(N):
    bonds = [1] + [3] * (N - 1) + [1]
    A, B = gen_tto_tto(seed=N, N=N, bonds=bonds, d1=2, d2=2, d3=3)
    ref = tomat(A) @ tomat(B)
    p = _mpo_params(A, B)
    for x in itertools.product(*[range(1, 7)] * N):
        assert O.feval(F_MPO, p, [6] * N, list(x)) == pytest.approx(
            fused_index_value(ref, x, [2] * N, [3] * N), rel=1e-12, abs=1e-13)


def test_oracle_batcheval_mpo_split():
    """_batchevaluate_dispatch over the contraction: every (row legs, column legs) split."""
    A, B = gen_tto_tto(seed=3)
    p = _mpo_params(A, B)
    ld = [4] * 4
    rng = np.random.default_rng(7)
    for nl in range(0, 5):
        I = rng.integers(1, 5, size=(5, nl))
        J = rng.integers(1, 5, size=(3, 4 - nl))
        out, _ = O.batcheval(F_MPO, p, ld, I, J, 0)
        for a in range(5):
            for b in range(3):
                x = list(I[a]) + list(J[b])
                assert out[a, 0, b] == O.feval(F_MPO, p, ld, x)


def test_contract_naive_is_matrix_product():
    A, B = gen_tto_tto(seed=1)
    ab = contract_naive(A, B)
    assert [list(c.shape[1:3]) for c in ab] == [[2, 2]] * 4  # sitedims (test_contraction.jl:92)
    np.testing.assert_allclose(tomat(ab), tomat(A) @ tomat(B), rtol=1e-12)


def test_contractsitetensors_layout():
    """_contractsitetensors (contraction.jl:591-602): fused bonds with A's index fastest."""
    rng = np.random.default_rng(2)
    a = rng.random((2, 3, 4, 5))
    b = rng.random((3, 4, 2, 2))
    c = _contractsitetensors(a, b)
    assert c.shape == (6, 3, 2, 10)
    for la, lb, s1, s3, ra, rb in itertools.product(range(2), range(3), range(3), range(2), range(5), range(2)):
        want = sum(a[la, s1, s2, ra] * b[lb, s2, s3, rb] for s2 in range(4))
        assert c[la + 2 * lb, s1, s3, ra + 5 * rb] == pytest.approx(want, rel=1e-14)


def test_mpo_mps_naive():
    rng = np.random.default_rng(4)
    bonds = [1, 2, 3, 2, 1]
    A = [rng.random((bonds[n], 3, 3, bonds[n + 1])) for n in range(4)]
    b = [rng.random((bonds[n], 3, bonds[n + 1])) for n in range(4)]
    ab = contract_naive(A, _as_mpo_right(b))
    v = tovec([np.reshape(c, (c.shape[0], c.shape[1] * c.shape[2], c.shape[3]), order="F") for c in ab])
    np.testing.assert_allclose(v, tomat(A) @ tovec(b), rtol=1e-12)


def test_contract_argument_errors():
    A, B = gen_tto_tto()
    with pytest.raises(ValueError):
        contract_naive(A[:3], B)
    bad = [np.zeros((1, 2, 4, 1))] + B[1:]
    with pytest.raises(ValueError):
        contract_naive(A, bad)


def test_contract_zipup_svd_is_matrix_product():
    """test_contraction.jl:185-189 (method = :SVD; host LAPACK, no device call)."""
    from tci_amd.contraction import contract_zipup
    A, B = gen_tto_tto(seed=5)
    ab = contract_zipup(A, B, method="SVD")
    np.testing.assert_allclose(tomat(ab), tomat(A) @ tomat(B), rtol=1e-10, atol=1e-12)


def gen_complex_tto_tto(seed=0, N=4, bonds=(1, 2, 3, 2, 1), d1=2, d2=3, d3=2):
    """_gen_testdata_TTO_TTO (test_contraction.jl:31-50): rand(ComplexF64, ...) cores."""
    rng = np.random.default_rng(seed)
    c = lambda *s: rng.random(s) + 1j * rng.random(s)  # noqa: E731
    A = [c(bonds[n], d1, d2, bonds[n + 1]) for n in range(N)]
    B = [c(bonds[n], d2, d3, bonds[n + 1]) for n in range(N)]
    return A, B


def test_realified_complex_contraction_is_the_complex_product():
    """The identity the device's Contraction{ComplexF64} rests on (tci_amd.contraction._realify):
    with both operators realified (2x2 real blocks, bonds doubled; X_re, X_im real MPOs of Re X,
    Im X), Re(A B) = A_re B_re - A_im B_im and Im(A B) = A_im B_re + A_re B_im, each a REAL MPO
    contraction."""
    from tci_amd.contraction import _realify
    for N, bonds in ((4, (1, 2, 3, 2, 1)), (1, (1, 1)), (2, (1, 3, 1))):
        A, B = gen_complex_tto_tto(seed=N, N=N, bonds=bonds)
        ref = tomat(A) @ tomat(B)
        Are, Aim = _realify(A)
        Br, Bi = _realify(B)
        np.testing.assert_allclose(tomat(Are) + 1j * tomat(Aim), tomat(A), rtol=1e-13, atol=1e-14)
        re = tomat(Are) @ tomat(Br) - tomat(Aim) @ tomat(Bi)
        im = tomat(Aim) @ tomat(Br) + tomat(Are) @ tomat(Bi)
        np.testing.assert_allclose(re + 1j * im, ref, rtol=1e-13, atol=1e-13)
        # ... and the oracle's real MPO evaluation of one part agrees with it
        p = _mpo_params(Are, Br)
        X = np.array(list(itertools.product(*[range(1, 5)] * N))[:40], np.int32)
        vals = np.array([O.feval(F_MPO, p, [4] * N, x) for x in X])
        want = np.array([fused_index_value(tomat(Are) @ tomat(Br), x, [2] * N, [2] * N) for x in X])
        np.testing.assert_allclose(vals, want, rtol=1e-13, atol=1e-14)


def test_complex_naive_and_zipup_svd():
    """contract(...; :naive) and :zipup (:SVD) of ComplexF64 operands (test_contraction.jl:68-98,
    185-195) are exact products on the host."""
    A, B = gen_complex_tto_tto(seed=3)
    ref = tomat(A) @ tomat(B)
    np.testing.assert_allclose(tomat(contract_naive(A, B)), ref, rtol=1e-12)
    from tci_amd.contraction import contract_zipup
    np.testing.assert_allclose(tomat(contract_zipup(A, B, method="SVD")), ref, rtol=1e-10, atol=1e-12)
