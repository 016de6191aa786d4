"""fp64 MFMA dense algebra (tci_dense.hip), through the C ABI:

* K3 `tci_dgemm_d` / `tci_schur_update_d` against numpy fp64 (ragged tiles, k = 0, k not a
  multiple of the 16-deep LDS stage, B and B^T), tolerance |err| <= 4 k eps sum|a||b| per entry
  (MFMA accumulates with one rounding per fused step, numpy/OpenBLAS in its own blocked order);
* K5 the blocked getrf/getrs of setsitetensor!'s solve `T = Pi1 * P^-1` (tensorci2.jl:620-627)
  at r in {256, 1024} against the oracle's loop-order restatement (rtol 1e-10, the site-tensor
  bar of DESIGN.md section 3);
* K4 MatrixLUCI factors with np in {256, 1024} (matrixluci.jl:161-241) against the oracle at
  rtol 1e-12 (pivots bitwise: the rrLU is unchanged).
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


def _dev(ctx, A, tight=False):
    A = np.asarray(A, dtype=np.float64)
    return T.DeviceMatrix(A.shape[0], A.shape[1], ctx=ctx, ld=A.shape[0] if tight else None).upload(A)


def _bound(A, B, k):
    return 4 * max(k, 1) * np.finfo(float).eps * (np.abs(A) @ np.abs(B)) + 1e-300


@pytest.mark.parametrize("m,n,k", [(1, 1, 1), (17, 33, 5), (200, 130, 64), (1000, 700, 37), (129, 257, 0),
                                   (2100, 1500, 100)])
@pytest.mark.parametrize("transb", [False, True])
def test_dgemm_vs_numpy(ctx, m, n, k, transb):
    rng = np.random.default_rng(m * 7 + n + k)
    A = rng.standard_normal((m, max(k, 1)))[:, :k]
    Bop = rng.standard_normal((max(k, 1), n))[:k, :]
    C0 = rng.standard_normal((m, n))
    dA = _dev(ctx, A) if k else T.DeviceMatrix(m, 1, ctx=ctx)
    dB = _dev(ctx, Bop.T if transb else Bop) if k else T.DeviceMatrix(max(n, 1), 1, ctx=ctx)
    dC = _dev(ctx, C0)
    alpha, beta = -1.25, 0.5
    T.dgemm_device(dA, dB, dC, alpha=alpha, beta=beta, transb=transb, k=k)
    got = dC.to_host()
    want = beta * C0 + alpha * (A @ Bop)
    err = np.abs(got - want)
    assert np.all(err <= abs(alpha) * _bound(A, Bop, k) + 4 * np.finfo(float).eps * np.abs(want)), err.max()


def test_schur_update_k3(ctx):
    # the standalone K3 shape of BASELINE.md:46 at a reduced size: C -= W V, nb = 256
    rng = np.random.default_rng(3)
    m, n, nb = 1536, 1280, 256
    C0, W, V = rng.random((m, n)), rng.random((m, nb)), rng.random((nb, n))
    dC = _dev(ctx, C0)
    T.schur_update_device(dC, _dev(ctx, W), _dev(ctx, V))
    got = dC.to_host()
    want = C0 - W @ V
    assert np.all(np.abs(got - want) <= _bound(W, V, nb) + 4 * np.finfo(float).eps * np.abs(C0)), \
        np.abs(got - want).max()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("r,R", [(256, 8192), (1024, 4096), (333, 1000), (70, 2000)])
def test_sitetensor_solve_mfma(ctx, r, R):
    rng = np.random.default_rng(r * 11 + R)
    # pivot matrices of a TCI are well conditioned by construction (maxvol-like pivots); a
    # diagonally weighted random matrix stands in for one, with partial pivoting still exercised
    P = rng.random((r, r)) + 0.5 * np.sqrt(r) * np.eye(r) * rng.choice([-1, 1], r)
    Pi1 = rng.random((R, r))
    ref = O.sitetensor_solve(P, Pi1).reshape((R, r), order="F")
    dP, dPi1, dT = _dev(ctx, P, True), _dev(ctx, Pi1, True), T.DeviceMatrix(R, r, ctx=ctx, ld=R)
    T.sitetensor_solve_device(dP, dPi1, dT)
    got = dT.to_host()
    np.testing.assert_allclose(got, ref, rtol=1e-10, atol=1e-12 * np.abs(ref).max())
    # the host entry takes the same path
    T_ = np.zeros(R * r)
    ctx.check(ctx.lib.tci_sitetensor_solve_h(ctx.h, T._lib.ptr(np.asfortranarray(P).ravel(order="F")), r,
                                             T._lib.ptr(np.asfortranarray(Pi1).ravel(order="F")), R,
                                             T._lib.ptr(T_)))
    np.testing.assert_allclose(T_.reshape((R, r), order="F"), ref, rtol=1e-10, atol=1e-12 * np.abs(ref).max())


@pytest.mark.timeout(300)
@pytest.mark.parametrize("r,R", [(1024, 256), (1500, 64), (97, 300), (24, 50), (2100, 16)])
def test_getrf_register_panel_bitwise(ctx, r, R):
    """The getrf panels held in registers (k_getrf_panel_reg, dense mask bit 8) against the LDS panel
    kernel (mask 7) and the oracle. Inside a panel both do the same arithmetic (true division,
    separate multiply and subtract, the first maximal |a| pivot), but the panel widths differ (24 /
    16 in registers, 16-64 in LDS), so the K3 trailing updates sum in a different blocking: equal to
    rounding, both within the parity tolerance of the oracle. r = 1500 runs two rows per thread,
    r = 2100 the LDS form for its first panels."""
    rng = np.random.default_rng(r + 7 * R)
    P = rng.random((r, r)) + 0.5 * np.sqrt(r) * np.eye(r) * rng.choice([-1, 1], r)
    Pi1 = rng.random((R, r))
    out = {}
    try:
        for mask in (15, 7):
            ctx.check(ctx.lib.tci_set_dense_mfma(ctx.h, mask))
            dP, dPi1, dT = _dev(ctx, P, True), _dev(ctx, Pi1, True), T.DeviceMatrix(R, r, ctx=ctx, ld=R)
            T.sitetensor_solve_device(dP, dPi1, dT)
            out[mask] = dT.to_host()
    finally:
        ctx.check(ctx.lib.tci_set_dense_mfma(ctx.h, 31))
    ref = O.sitetensor_solve(P, Pi1).reshape((R, r), order="F")
    np.testing.assert_allclose(out[15], out[7], rtol=1e-11, atol=1e-13 * np.abs(ref).max())
    np.testing.assert_allclose(out[15], ref, rtol=1e-10, atol=1e-12 * np.abs(ref).max())


@pytest.mark.timeout(300)
@pytest.mark.parametrize("r,R", [(1024, 4096), (1000, 300), (256, 2048), (97, 300), (70, 130), (24, 50),
                                 (8, 9), (1, 5), (1100, 40)])
def test_sitetensor_solve_coop_recursive(ctx, r, R):
    """Round 6: the cooperative one-launch getrf (mask bit 16, r <= 1024) against the
    launch-per-panel form (mask 15), the LDS panels (7) and the oracle. Every form factorises with
    the same pivot rule; the sums run in other orders, so they agree to rounding. r = 1100 is past
    the cooperative kernel's 1024 rows (the blocked getrf runs)."""
    rng = np.random.default_rng(r * 5 + R)
    P = rng.random((r, r)) + 0.5 * np.sqrt(r) * np.eye(r) * rng.choice([-1, 1], r)
    Pi1 = rng.random((R, r))
    ref = O.sitetensor_solve(P, Pi1).reshape((R, r), order="F")
    out = {}
    try:
        for mask in (31, 15, 7):
            ctx.check(ctx.lib.tci_set_dense_mfma(ctx.h, mask))
            dP, dPi1, dT = _dev(ctx, P, True), _dev(ctx, Pi1, True), T.DeviceMatrix(R, r, ctx=ctx, ld=R)
            T.sitetensor_solve_device(dP, dPi1, dT)
            out[mask] = dT.to_host()
    finally:
        ctx.check(ctx.lib.tci_set_dense_mfma(ctx.h, 31))
    tol = dict(rtol=1e-10, atol=1e-12 * np.abs(ref).max())
    for mask, got in out.items():
        np.testing.assert_allclose(got, ref, err_msg=f"mask {mask}", **tol)
        np.testing.assert_allclose(got, out[15], err_msg=f"mask {mask} vs 15", **tol)


@pytest.mark.timeout(300)
@pytest.mark.parametrize("r,R", [(256, 512), (1024, 96)])
def test_coop_getrf_fault_falls_back(ctx, monkeypatch, r, R):
    """The cooperative getrf's give-up path (a workgroup waited past its timeout: every workgroup
    leaves and sets the fault word), simulated by TCI_COOP_FAULT_TEST=1: solve_launch reads the
    word, restores P from its copy and redoes the solve on the launch-per-panel path -- so the
    result is bitwise that path's (mask 15), and the context keeps working afterwards."""
    rng = np.random.default_rng(r + 3 * R)
    P = rng.random((r, r)) + 0.5 * np.sqrt(r) * np.eye(r) * rng.choice([-1, 1], r)
    Pi1 = rng.random((R, r))

    def solve(mask):
        ctx.check(ctx.lib.tci_set_dense_mfma(ctx.h, mask))
        dP, dPi1, dT = _dev(ctx, P, True), _dev(ctx, Pi1, True), T.DeviceMatrix(R, r, ctx=ctx, ld=R)
        T.sitetensor_solve_device(dP, dPi1, dT)
        return dT.to_host()

    try:
        monkeypatch.setenv("TCI_COOP_FAULT_TEST", "1")
        fell_back = solve(31)
        monkeypatch.delenv("TCI_COOP_FAULT_TEST")
        blocked = solve(15)
        coop = solve(31)
    finally:
        ctx.check(ctx.lib.tci_set_dense_mfma(ctx.h, 31))
    assert np.array_equal(fell_back, blocked)
    ref = O.sitetensor_solve(P, Pi1).reshape((R, r), order="F")
    np.testing.assert_allclose(coop, ref, rtol=1e-10, atol=1e-12 * np.abs(ref).max())


@pytest.mark.timeout(300)
@pytest.mark.parametrize("r", [256, 1024])
def test_sitetensor_solve_unweighted_backward_error(ctx, r):
    """A plain U[0,1) pivot matrix (no diagonal weight: cond ~ 1e4-1e6, partial pivoting with real
    row exchanges everywhere): the default solve's backward error ||T P - Pi1|| / (||T|| ||P||) stays
    at the level of a LAPACK solve's, and it agrees with the launch-per-panel / left-looking forms to cond(P) eps."""
    rng = np.random.default_rng(r + 1)
    P = rng.random((r, r))
    R = 3 * r
    Pi1 = rng.random((R, r))
    got = {}
    try:
        for mask in (31, 15):
            ctx.check(ctx.lib.tci_set_dense_mfma(ctx.h, mask))
            dP, dPi1, dT = _dev(ctx, P, True), _dev(ctx, Pi1, True), T.DeviceMatrix(R, r, ctx=ctx, ld=R)
            T.sitetensor_solve_device(dP, dPi1, dT)
            got[mask] = dT.to_host()
    finally:
        ctx.check(ctx.lib.tci_set_dense_mfma(ctx.h, 31))
    eps = np.finfo(float).eps
    for mask, Tm in got.items():
        berr = np.linalg.norm(Tm @ P - Pi1) / (np.linalg.norm(Tm) * np.linalg.norm(P))
        assert berr < 64 * r * eps, (mask, berr)
    cond = np.linalg.cond(P)
    assert np.linalg.norm(got[31] - got[15]) <= 64 * r * eps * cond * np.linalg.norm(got[15])


@pytest.mark.timeout(300)
@pytest.mark.parametrize("np_", [256, 1024])
@pytest.mark.parametrize("leftorth", [True, False])
def test_luci_factors_mfma(ctx, np_, leftorth):
    A = O.fill_uniform(2304 * 1792, 21).reshape((2304, 1792), order="F")
    luci = T.MatrixLUCI(A, maxrank=np_, leftorthogonal=leftorth, ctx=ctx)
    ref = O.OracleLU(A, maxrank=np_, leftorthogonal=leftorth)
    assert np.array_equal(luci.rowindices() - 1, ref.rowindices())
    assert np.array_equal(luci.colindices() - 1, ref.colindices())
    np.testing.assert_allclose(luci.left(), ref.left, rtol=1e-12, atol=1e-12 * np.abs(ref.left).max())
    np.testing.assert_allclose(luci.right(), ref.right, rtol=1e-12, atol=1e-12 * np.abs(ref.right).max())
