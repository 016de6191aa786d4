"""CPU check of the certified shadow search's error bound (tci_rrlu.hip
k_pass_mf, tci_rrlu_c128.hip k_crrlu_step_sh): the fp16 shadow of the stale values, scaled per
epoch, minus the pending rank-1 updates as f16 two-term splits accumulated in fp32 must stay within
the eps the kernels use of the exact (scaled) value, for every trailing element -- otherwise the
search could skip the argmax. The data are genuine full-pivoting LU states (numpy restatement of
_optimizerrlu! steps, matrixlu.jl:46-87, 295-322), so |stale| <= |pivot t0| and |x_s y_s| <=
|pivot_s| hold as in the kernels. fp32 accumulation is emulated in two orders (sequential and
pairwise); the MFMA's internal order is not specified, the bound covers any order."""
import math

import numpy as np
import pytest


def f16(v):
    return np.asarray(v, np.float32).astype(np.float16)


def split(v):
    hi = f16(np.asarray(v, np.float64).astype(np.float32))
    lo = f16((np.asarray(v, np.float64) - hi.astype(np.float64)).astype(np.float32))
    return hi.astype(np.float32), lo.astype(np.float32)


def sh_scale(B):
    if not (2.0 ** -100 <= B <= 2.0 ** 100):
        return 0.0
    return math.ldexp(1.0, 14 - (math.frexp(B)[1] - 1))


def lu_states(A, steps):
    """Full pivoting with the reference's order; yields (pivot values, x's, y's, trailing stale
    block after step t0 - 1 for every t0) -- leftorth: x = column / pivot, y = row."""
    A = A.copy()
    m, n = A.shape
    rows, cols = np.arange(m), np.arange(n)
    piv, X, Y, blocks = [], [], [], []
    for k in range(steps):
        blocks.append((A.copy(), rows.copy(), cols.copy()))
        sub = np.abs(A) ** 2
        j = int(np.argmax(sub.max(axis=0)))
        i = int(np.argmax(sub[:, j]))
        p = A[i, j]
        x = A[:, j] / p
        y = A[i, :].copy()
        piv.append(p)
        X.append((x, rows.copy()))
        Y.append((y, cols.copy()))
        A = A - np.outer(x, y)
        A = np.delete(np.delete(A, i, 0), j, 1)
        rows = np.delete(rows, i)
        cols = np.delete(cols, j)
    return piv, X, Y, blocks


def restrict(vec_rows, rows):
    v, r = vec_rows
    pos = {int(q): a for a, q in enumerate(r)}
    return np.array([v[pos[int(q)]] for q in rows])


@pytest.mark.parametrize("seed,decay", [(0, 0.0), (1, 0.3), (2, 0.0)])
def test_real_mfma_shadow_bound(seed, decay):
    rng = np.random.default_rng(seed)
    m, n = 160, 140
    A = rng.random((m, n)) - 0.3
    if decay:
        A = A * np.exp(-decay * np.arange(n))[None, :]
    piv, X, Y, blocks = lu_states(A, 20)
    worst = 0.0
    for t0 in (0, 1, 3):
        stale, rows0, cols0 = blocks[t0]
        pv = np.abs(np.array(piv))
        B = pv[0] if t0 == 0 else 2.0 * pv[t0 - 1]
        s = sh_scale(B)
        h = f16((stale * s).astype(np.float32)).astype(np.float32)
        for P in range(1, 16):  # P <= 10: one MFMA K-step, 11..15: two
            k = t0 + P - 1
            stale_k, rows_k, cols_k = blocks[k + 1] if k + 1 < len(blocks) else (None, None, None)
            if stale_k is None:
                break
            # exact trailing values after pivots t0..k, restricted to the rows / columns still in
            ri = [int(np.where(rows0 == q)[0][0]) for q in rows_k]
            ci = [int(np.where(cols0 == q)[0][0]) for q in cols_k]
            W1 = h[np.ix_(ri, ci)].astype(np.float32).copy()
            terms = []
            for q in range(P):
                xs = restrict(X[t0 + q], rows_k)
                ys = restrict(Y[t0 + q], cols_k) * s
                xh, xl = split(-xs)
                yh, yl = split(ys)
                terms += [np.outer(xh, yh), np.outer(xh, yl), np.outer(xl, yh)]
            for tm in terms:  # sequential fp32 accumulation
                W1 = (W1 + tm.astype(np.float32)).astype(np.float32)
            W2 = h[np.ix_(ri, ci)].astype(np.float32) + np.sum(np.array(terms, np.float32), axis=0, dtype=np.float32)
            exact = stale_k * s
            Mf, sumM = pv[t0], pv[t0:t0 + P].sum()
            mag = Mf + 2.0 * sumM
            eps = (2.0 ** -11 * (1 + 2.0 ** -9) * Mf * s + 2.0 ** -25 + 2.0 ** -19 * sumM * s + P * 2.0 ** -24
                   + (3 * P + 4) * 2.0 ** -23 * mag * s)
            err = max(np.abs(W1 - exact).max(), np.abs(W2 - exact).max())
            worst = max(worst, err / eps)
    assert worst < 1.0, worst
    assert worst > 1e-3  # the bound is not vacuous


def test_complex_mfma_shadow_bound():
    rng = np.random.default_rng(7)
    m, n = 120, 110
    A = (rng.random((m, n)) - 0.5) + 1j * (rng.random((m, n)) - 0.5)
    piv, X, Y, blocks = lu_states(A, 12)
    pv = np.abs(np.array(piv))
    worst = 0.0
    for t0 in (0, 2):
        stale, rows0, cols0 = blocks[t0]
        B = pv[0] if t0 == 0 else 2.0 * pv[t0 - 1]
        s = sh_scale(B)
        hr = f16((stale.real * s).astype(np.float32)).astype(np.float32)
        hi = f16((stale.imag * s).astype(np.float32)).astype(np.float32)
        for P in range(1, 11):
            k = t0 + P - 1
            if k + 1 >= len(blocks):
                break
            stale_k, rows_k, cols_k = blocks[k + 1]
            ri = [int(np.where(rows0 == q)[0][0]) for q in rows_k]
            ci = [int(np.where(cols0 == q)[0][0]) for q in cols_k]
            Wr = hr[np.ix_(ri, ci)].copy()
            Wi = hi[np.ix_(ri, ci)].copy()
            for q in range(P):
                xs = -restrict(X[t0 + q], rows_k)
                ys = restrict(Y[t0 + q], cols_k) * s
                xrh, xrl = split(xs.real)
                xih, xil = split(xs.imag)
                yrh, yrl = split(ys.real)
                yih, yil = split(ys.imag)
                nyih, nyil = split(-ys.imag)
                # slots (xr_h,xr_h,xr_l,xi_h,xi_h,xi_l) x re-plane (yr_h,yr_l,yr_h,-yi_h,-yi_l,-yi_h)
                for a, b in ((xrh, yrh), (xrh, yrl), (xrl, yrh), (xih, nyih), (xih, nyil), (xil, nyih)):
                    Wr = (Wr + np.outer(a, b).astype(np.float32)).astype(np.float32)
                # and x im-plane (yi_h,yi_l,yi_h,yr_h,yr_l,yr_h)
                for a, b in ((xrh, yih), (xrh, yil), (xrl, yih), (xih, yrh), (xih, yrl), (xil, yrh)):
                    Wi = (Wi + np.outer(a, b).astype(np.float32)).astype(np.float32)
            exact = stale_k * s
            Mf, sumM = pv[t0], pv[t0:t0 + P].sum()
            mag = Mf + 2.0 * sumM
            epsc = (2.0 ** -11 * (1 + 2.0 ** -9) * Mf * s + 2.0 ** -25 + 2.0 ** -18 * sumM * s
                    + 2 * P * 2.0 ** -24 + (6 * P + 4) * 2.0 ** -23 * mag * s)
            epsd = math.sqrt(2.0) * (1 + 2.0 ** -20) * epsc + 2.0 ** -21 * mag * s
            mod = np.sqrt((Wr.astype(np.float32) ** 2 + Wi.astype(np.float32) ** 2).astype(np.float32))
            err = np.abs(mod - np.abs(exact)).max()
            worst = max(worst, err / epsd)
    assert worst < 1.0, worst
    assert worst > 1e-3
