"""GPU parity of the contraction evaluator (TCI_F_MPO: k_mpo_env environments + fp64 MFMA GEMM)
and of contract(A, B; algorithm=:TCI) (contraction.jl:483-575, 692-732, 832-891).

Bars: batch evaluation within 1e-12 relative of the oracle (summation order of the environments
and of the GEMM differs from the per-point chain); TCI2 over the contraction: ranks equal to the
oracle's and errors within 1e-10 relative (north star); contract(...; :TCI) reproduces the
matrix product of the operands (the reference's own test, test_contraction.jl:94, 175) within
1e-10 relative to its largest entry.
"""
import itertools

import numpy as np
import pytest

import oracle_lib as O
from test_contraction_oracle import F_MPO, fused_index_value, gen_tto_tto

pytestmark = pytest.mark.gpu

T = pytest.importorskip("tci_amd")
from tci_amd.contraction import _mpo_params, tomat, tovec  # noqa: E402


@pytest.fixture(scope="module")
def ctx():
    c = T.Context(0)
    yield c
    c.close()


def relerr(a, b):
    return np.abs(np.asarray(a) - np.asarray(b)).max() / max(np.abs(b).max(), 1e-300)


@pytest.mark.parametrize("M", [0, 1])
def test_batcheval_vs_oracle_every_split(ctx, M):
    A, B = gen_tto_tto(seed=11)
    f = T.Contraction(A, B, ctx=ctx)
    p = _mpo_params(A, B)
    rng = np.random.default_rng(5)
    for nl in range(0, 5 - M):
        I = rng.integers(1, 5, size=(7, nl)).astype(np.int32)
        J = rng.integers(1, 5, size=(6, 4 - nl - M)).astype(np.int32)
        got, mx = f.pi(I, J, M)
        ref, rmx = O.batcheval(F_MPO, p, [4] * 4, I, J, M)
        ref = ref.reshape(got.shape, order="F")
        assert relerr(got, ref) <= 1e-12
        assert mx == pytest.approx(rmx, rel=1e-12)


def test_points_are_the_matrix_product(ctx):
    A, B = gen_tto_tto(seed=12)
    f = T.Contraction(A, B, ctx=ctx)
    ref = tomat(A) @ tomat(B)
    X = np.array(list(itertools.product(*[range(1, 5)] * 4)), np.int32)
    got = f.points(X)
    want = np.array([fused_index_value(ref, x, [2] * 4, [2] * 4) for x in X])
    assert relerr(got, want) <= 1e-12


def test_larger_bonds_vs_oracle(ctx):
    """bond dimension 24 (K = 576 environment terms, the LDS-tiled MFMA GEMM), 10 sites."""
    N, chi = 10, 24
    bonds = [1] + [chi] * (N - 1) + [1]
    A, B = gen_tto_tto(seed=13, N=N, bonds=bonds, d1=2, d2=2, d3=2)
    f = T.Contraction(A, B, ctx=ctx)
    p = _mpo_params(A, B)
    rng = np.random.default_rng(6)
    I = rng.integers(1, 5, size=(200, 5)).astype(np.int32)
    J = rng.integers(1, 5, size=(150, 5)).astype(np.int32)
    got, _ = f.pi(I, J, 0)
    ref, _ = O.batcheval(F_MPO, p, [4] * N, I, J, 0)
    assert relerr(got, ref.reshape(got.shape, order="F")) <= 1e-12


def test_tci2_over_contraction_vs_oracle(ctx):
    A, B = gen_tto_tto(seed=14)
    f = T.Contraction(A, B, ctx=ctx)
    p = _mpo_params(A, B)
    piv = [T.optfirstpivot(f, f.localdims, [1] * 4)]
    kw = dict(tolerance=1e-12, maxiter=8)
    tci, ranks, errors = T.crossinterpolate2(f, f.localdims, piv, nsearchglobalpivot=0, **kw)
    rt, rranks, rerrors = O.crossinterpolate2(F_MPO, p, [4] * 4, piv, **kw)
    assert ranks == rranks
    np.testing.assert_allclose(errors, rerrors, rtol=1e-10, atol=1e-14)


def test_contract_tci_is_matrix_product(ctx):
    """test_contraction.jl:86-98 (f = nothing, algorithm = :TCI)."""
    A, B = gen_tto_tto(seed=15)
    ab = T.contract(A, B, algorithm="TCI", seed=0, ctx=ctx)
    assert [list(c.shape[1:3]) for c in ab] == [[2, 2]] * 4
    ref = tomat(A) @ tomat(B)
    assert relerr(tomat(ab), ref) <= 1e-10


def test_contract_mpo_mps(ctx):
    """test_contraction.jl:148-182: MPO x MPS and MPS x MPO."""
    rng = np.random.default_rng(16)
    bonds = [1, 2, 3, 2, 1]
    A = [rng.random((bonds[n], 3, 3, bonds[n + 1])) for n in range(4)]
    b = [rng.random((bonds[n], 3, bonds[n + 1])) for n in range(4)]
    ab = T.contract(A, b, seed=0, ctx=ctx)
    ba = T.contract(b, A, seed=0, ctx=ctx)
    assert [c.shape[1] for c in ab] == [3] * 4
    assert relerr(tovec(ab), tomat(A) @ tovec(b)) <= 1e-10
    assert relerr(tovec(ba), tovec(b) @ tomat(A)) <= 1e-10


def test_contract_naive_matches_tci(ctx):
    A, B = gen_tto_tto(seed=17)
    assert relerr(tomat(T.contract(A, B, algorithm="TCI", seed=1, ctx=ctx)),
                  tomat(T.contract(A, B, algorithm="naive"))) <= 1e-10


def test_contraction_argument_errors(ctx):
    A, B = gen_tto_tto()
    with pytest.raises(ValueError):
        T.Contraction(A[:3], B, ctx=ctx)
    with pytest.raises(ValueError):
        T.contract(A, B, algorithm="bogus", ctx=ctx)
    with pytest.raises(RuntimeError):
        T.contract(A, B, algorithm="naive", f=lambda x: 2 * x)
    big = 64  # ra * rb = 4096 > the environment kernel's 2048
    A2, B2 = gen_tto_tto(seed=2, N=3, bonds=[1, big, big, 1], d1=2, d2=2, d3=2)
    with pytest.raises(T.TCIArgumentError):
        T.Contraction(A2, B2, ctx=ctx)


@pytest.mark.parametrize("method", ["LU", "CI"])
def test_contract_zipup_device_factorizations(ctx, method):
    """test_contraction.jl:185-195: zip-up with the rrLU / MatrixLUCI factorizations (device)."""
    A, B = gen_tto_tto(seed=18)
    ab = T.contract(A, B, algorithm="zipup", method=method, ctx=ctx)
    assert relerr(tomat(ab), tomat(A) @ tomat(B)) <= 1e-10
    rng = np.random.default_rng(19)
    bonds = [1, 2, 3, 2, 1]
    A3 = [rng.random((bonds[n], 3, 3, bonds[n + 1])) for n in range(4)]
    b = [rng.random((bonds[n], 3, bonds[n + 1])) for n in range(4)]
    ab3 = T.contract(A3, b, algorithm="zipup", method=method, ctx=ctx)
    assert relerr(tovec(ab3), tomat(A3) @ tovec(b)) <= 1e-10


# ------------------------------------------------------------------ ComplexF64 and the elementwise f
from test_contraction_oracle import gen_complex_tto_tto  # noqa: E402


def _tto_tts_complex(seed):
    """_gen_testdata_TTO_TTS (test_contraction.jl:52-66): ComplexF64 MPO (3 x 3 legs) and MPS."""
    rng = np.random.default_rng(seed)
    c = lambda *s: rng.random(s) + 1j * rng.random(s)  # noqa: E731
    bonds = [1, 2, 3, 2, 1]
    A = [c(bonds[n], 3, 3, bonds[n + 1]) for n in range(4)]
    b = [c(bonds[n], 3, bonds[n + 1]) for n in range(4)]
    return A, b


@pytest.mark.parametrize("M", [0, 1])
def test_complex_batcheval_is_the_complex_product(ctx, M):
    """Contraction{ComplexF64} batches (four real MPO contractions on the device, summed into the
    complex Pi by TCI_F_C128) against the complex matrix product, at every split of the legs."""
    A, B = gen_complex_tto_tto(seed=21)
    f = T.Contraction(A, B, ctx=ctx)
    assert f.is_complex
    ref = tomat(A) @ tomat(B)
    rng = np.random.default_rng(22)
    for nl in range(0, 5 - M):
        I = rng.integers(1, 5, size=(7, nl)).astype(np.int32)
        J = rng.integers(1, 5, size=(6, 4 - nl - M)).astype(np.int32)
        got, mx = f.pi(I, J, M)
        D = 4 if M else 1
        want = np.zeros((7 * D, 6), np.complex128)
        for i in range(7):
            for c in range(D):
                for j in range(6):
                    x = list(I[i]) + ([c + 1] if M else []) + list(J[j])
                    want[i + 7 * c, j] = fused_index_value(ref, x, [2] * 4, [2] * 4)
        assert relerr(got, want) <= 1e-12
        assert mx == pytest.approx(np.abs(want).max(), rel=1e-12)


@pytest.mark.parametrize("f", [None, "2x"])
@pytest.mark.parametrize("algorithm", ["TCI", "naive"])
def test_complex_mpo_mpo_contraction(ctx, f, algorithm):
    """The reference's "MPO-MPO contraction" testset (test_contraction.jl:68-98): ComplexF64
    operands, f in [nothing, x -> 2x], algorithm in [:TCI, :naive]; :naive with f throws."""
    fn = (lambda x: 2 * x) if f else None
    A, B = gen_complex_tto_tto(seed=23)
    if fn is not None and algorithm == "naive":
        with pytest.raises(RuntimeError):
            T.contract(A, B, f=fn, algorithm=algorithm)
        return
    ab = T.contract(A, B, f=fn, algorithm=algorithm, seed=0, ctx=ctx)
    assert [list(c.shape[1:3]) for c in ab] == [[2, 2]] * 4
    ref = tomat(A) @ tomat(B)
    if fn is not None:
        ref = fn(ref)
    assert relerr(tomat(ab), ref) <= 1e-10


@pytest.mark.parametrize("f", [None, "2x"])
def test_complex_mpo_mps_contraction(ctx, f):
    """The reference's "MPO-MPS contraction" testset (test_contraction.jl:148-183), :TCI."""
    fn = (lambda x: 2 * x) if f else None
    A, b = _tto_tts_complex(seed=24)
    ab = T.contract(A, b, f=fn, seed=0, ctx=ctx)
    ba = T.contract(b, A, f=fn, seed=0, ctx=ctx)
    assert [c.shape[1] for c in ab] == [3] * 4
    want_ab = tomat(A) @ tovec(b)
    want_ba = tovec(b) @ tomat(A)
    if fn is not None:
        want_ab, want_ba = fn(want_ab), fn(want_ba)
    assert relerr(tovec(ab), want_ab) <= 1e-10
    assert relerr(tovec(ba), want_ba) <= 1e-10


def test_real_contraction_with_f(ctx):
    """Contraction(A, B; f) for Float64 operands: f on the host over the device products, the
    factorisation on the device (test_contraction.jl:68 with f = x -> 2x; and a nonlinear f)."""
    A, B = gen_tto_tto(seed=25)
    ab = T.contract(A, B, f=lambda x: 2 * x, seed=0, ctx=ctx)
    assert relerr(tomat(ab), 2 * (tomat(A) @ tomat(B))) <= 1e-10
    g = T.Contraction(A, B, ctx=ctx, f=np.sin)
    X = np.array(list(itertools.product(*[range(1, 5)] * 4))[:50], np.int32)
    ref = tomat(A) @ tomat(B)
    want = np.sin([fused_index_value(ref, x, [2] * 4, [2] * 4) for x in X])
    assert relerr(g.points(X), want) <= 1e-12
    # a scalar-only f (math.sin refuses arrays) goes element by element
    import math
    h = T.Contraction(A, B, ctx=ctx, f=math.sin)
    assert relerr(h.points(X), want) <= 1e-12


@pytest.mark.parametrize("method", ["LU", "SVD"])
def test_complex_zipup(ctx, method):
    """test_contraction.jl:185-195 on ComplexF64 operands (:LU = the device complex rrLU)."""
    A, B = gen_complex_tto_tto(seed=26)
    ab = T.contract(A, B, algorithm="zipup", method=method, ctx=ctx)
    assert relerr(tomat(ab), tomat(A) @ tomat(B)) <= 1e-10
