"""CachedFunction host logic (tci_amd/cachedfunction.py) against the reference's own testset
(test/test_cachedfunction.jl). Host-only: the wrapped functions here are Python callables, as in
the reference; the device-evaluator case is in tests/test_gpu_complex.py."""
import numpy as np
import pytest

import tci_amd as T


@pytest.mark.parametrize("vt", [float, complex])
def test_cache(vt):  # test_cachedfunction.jl:50-58
    def f(x):
        return 2 * (x[0] - 1) + (x[1] - 1)

    cf = T.CachedFunction(f, [4, 2], vt)
    assert cf.f is f
    for i in range(1, 5):
        for j in range(1, 3):
            x = [i, j]
            assert cf(x) == f(x)
            assert cf.key(x) in cf.cache
            assert cf(x) == f(x)
    assert cf.ncacheddata() == 8
    assert cf.cacheddata()[(3, 2)] == f([3, 2])
    cf.clearcache()
    assert cf.ncacheddata() == 0


@pytest.mark.parametrize("vt", [float, complex])
def test_cache_batcheval(vt):  # :81-90
    localdims = [2, 2, 2, 2, 2]
    calls = []

    def f(x):
        calls.append(1)
        return sum(x)

    cf = T.CachedFunction(f, localdims, vt)
    left = [[1, 1]] * 100
    right = [[1, 1]] * 100
    res = cf(left, right, 1)
    ref = np.array([[[sum(lft + [c] + r) for r in right] for c in (1, 2)] for lft in left])
    assert res.shape == (100, 2, 100)
    np.testing.assert_array_equal(res, ref)
    assert len(calls) == 2  # repeated points are evaluated once
    cf(left, right, 1)
    assert len(calls) == 2


def test_many_bits():  # :92-100
    N = 64 * 4
    cf = T.CachedFunction(lambda x: 1.0, [2] * N)
    x = [1] * N
    assert cf(x) == 1.0 and cf.key(x) == 0
    assert cf.keytype == "UInt256+"
    y = [2] * N
    assert cf.key(y) == 2 ** N - 1
    np.testing.assert_array_equal(cf.points(np.array([x, y])), [1.0, 1.0])


def test_key_collision():  # :112-129 (1e4 samples; the memory-overhead bounds are Julia-specific)
    nbit = 36
    cf = T.CachedFunction(lambda x: 1.0, [2] * nbit, complex)
    for i in range(1, 10001):
        b = [((i - 1) >> (nbit - 1 - n) & 1) + 1 for n in range(nbit)]
        cf(b)
    assert cf.ncacheddata() == 10000


def test_key_boundary_check():  # :131-137
    cf = T.CachedFunction(lambda x: 1.0, [2] * 40, complex)
    with pytest.raises(ValueError):
        cf.key([1] * 80)


def test_pi_layout():
    # Pi element (i + m*c, j) = f([I_i..., c, J_j...]) with i fastest (batcheval.jl:157-171)
    cf = T.CachedFunction(lambda x: 100 * x[0] + 10 * x[1] + x[2], [3, 4, 5])
    I = np.array([[1], [3]])
    J = np.array([[2], [5], [4]])
    Pi, mx = cf.pi(I, J, 1)
    assert Pi.shape == (8, 3)
    for i in range(2):
        for c in range(4):
            for j in range(3):
                assert Pi[i + 2 * c, j] == 100 * I[i, 0] + 10 * (c + 1) + J[j, 0]
    assert mx == np.abs(Pi).max()
