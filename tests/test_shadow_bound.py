"""CPU check of the certified shadow search's error bound (tci_rrlu.hip
k_pass_mf, tci_rrlu_c128.hip k_crrlu_step_sh): the fp16 shadow (or, TCI_SH_U8, the 8-bit codes) of
the stale values, scaled per epoch, minus the pending rank-1 updates as f16 two-term splits accumulated in fp32 must stay within
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


def sh_scale(B, mode="f16"):
    if not (2.0 ** -100 <= B <= 2.0 ** 100):
        return 0.0
    if mode == "u8":
        return 127.0 / B  # tci_rrlu.hip sh_scale, TCI_SH_U8
    return math.ldexp(1.0, 13 - (math.frexp(B)[1] - 1))  # tci_rrlu.hip sh_scale (kShExp = 13)


def sh_rscale(B, mode="f16"):
    """tci_rrlu.hip sh_rscale: >= 1 / sh_scale(B)"""
    if mode == "u8":
        return B * (1.0 / 127.0) * (1.0 + 2.0 ** -40)
    return 1.0 / sh_scale(B)


def store(v_scaled, mode):
    """the shadow of scaled values as the kernels store it, read back as fp32 (u8: the decoded
    integer q; the kernels add the -128 offset inside the MFMA -- see accumulate)"""
    f = np.asarray(v_scaled, np.float32)
    if mode == "u8":
        return np.rint(np.clip(f, np.float32(-127), np.float32(127))).astype(np.float32)  # sh_u8
    return f16(f).astype(np.float32)


def accumulate(h, terms, mode, order):
    """fp32 accumulation of the shadow and the split-product terms (u8: from the byte q + 128 and
    the offset slot 1 x (-128), as the MFMA sees them), sequentially or pairwise"""
    h = np.asarray(h, np.float32)
    terms = [t.astype(np.float32) for t in terms]
    if mode == "u8":
        h = (h + np.float32(128)).astype(np.float32)
        terms = terms + [np.full(h.shape, -128.0, np.float32)]
    if order == "seq":
        W = h.copy()
        for tm in terms:
            W = (W + tm).astype(np.float32)
        return W
    return h + np.sum(np.array(terms, np.float32), axis=0, dtype=np.float32)


def eps_abs(mode, d, Mfd, sumM, P, rs):
    """tci_rrlu.hip sh_cert's per-epoch bound in absolute units"""
    mag = Mfd + 2.0 * sumM
    if mode == "u8":
        return (d + (0.5 + 2.0 ** -14) * rs + 2.0 ** -19 * sumM + P * 2.0 ** -24 * rs
                + (3 * P + 5) * 2.0 ** -23 * (mag + 384.0 * rs))
    return (d + 2.0 ** -11 * (1 + 2.0 ** -9) * Mfd + 2.0 ** -25 * rs + 2.0 ** -19 * sumM + P * 2.0 ** -24 * rs
            + (3 * P + 4) * 2.0 ** -23 * mag)


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


@pytest.mark.parametrize("mode", ["f16", "u8"])
@pytest.mark.parametrize("seed,decay", [(0, 0.0), (1, 0.3), (2, 0.0)])
def test_real_mfma_shadow_bound(seed, decay, mode):
    """f16: the fp16 shadow (default build); u8: the 8-bit codes of TCI_SH_U8 (clamped, rounded
    to an integer at s = 127 / B, widened into the accumulator with the -128 offset slot)."""
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
        s = sh_scale(B, mode)
        h = store((stale * s).astype(np.float32), mode)
        for P in range(1, 16):  # P <= 10: one MFMA K-step, 11..15: two
            k = t0 + P - 1
            stale_k, rows_k, cols_k = blocks[k + 1] if k + 1 < len(blocks) else (None, None, None)
            if stale_k is None:
                break
            # exact trailing values after pivots t0..k, restricted to the rows / columns still in
            ri = [int(np.where(rows0 == q)[0][0]) for q in rows_k]
            ci = [int(np.where(cols0 == q)[0][0]) for q in cols_k]
            terms = []
            for q in range(P):
                xs = restrict(X[t0 + q], rows_k)
                ys = restrict(Y[t0 + q], cols_k) * s
                xh, xl = split(-xs)
                yh, yl = split(ys)
                terms += [np.outer(xh, yh), np.outer(xh, yl), np.outer(xl, yh)]
            W1 = accumulate(h[np.ix_(ri, ci)], terms, mode, "seq")
            W2 = accumulate(h[np.ix_(ri, ci)], terms, mode, "pairwise")
            exact = stale_k * s
            Mf, sumM = pv[t0], pv[t0:t0 + P].sum()
            eps = eps_abs(mode, 0.0, Mf, sumM, P, sh_rscale(B, mode)) * s
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


def sh_cert(pv, k, PS, PE, nbs, tight=None, mode="f16"):
    """Python restatement of tci_rrlu.hip sh_cert (two-level epoch): (eps in absolute units,
    certified) of the shadow-search pass after pivot k."""
    if tight is None:
        tight = 4 if mode == "u8" else 7  # TCI_SH_TIGHT_U8 / TCI_SH_TIGHT
    te, t0 = k - PE + 1, k - PS + 1
    d = 0.0
    e = te
    while True:
        cur = e >= t0
        ke = k if cur else e + nbs - 1
        P = ke - e + 1
        sumM = float(np.sum(pv[e:ke + 1]))
        maxM = float(np.max(pv[e:ke + 1]))
        B = pv[0] if e == 0 else 2.0 * pv[e - 1]
        s = sh_scale(B, mode)
        Mfd = pv[e] + d
        mag = Mfd + 2.0 * sumM
        ea = eps_abs(mode, d, Mfd, sumM, P, sh_rscale(B, mode)) if s > 0 else 0.0
        ok = s > 0 and mag < 2.0 ** 100 and maxM * s <= 2.0 ** 15 and ea * s < math.ldexp(pv[ke] * s, -tight)
        if cur:
            return ea, ok
        d = ea if ok else 0.0
        e += nbs


@pytest.mark.parametrize("mode", ["f16", "u8"])
@pytest.mark.parametrize("seed,decay,nb", [(0, 0.0, 5), (1, 0.0, 10), (2, 0.02, 4), (3, 0.0, 3)])
def test_real_two_level_epoch_accumulated_bound(seed, decay, nb, mode):
    """The two-level epoch: each shadow epoch of nb pivots ends with a refresh that
    stores fl16(s_new / s_old W) -- W the MFMA search's fp32 value, not the exact one -- so the next
    epochs start from a shadow whose error against the exact stale values is the previous pass's
    whole bound. Emulated over 3 epochs (up to 3 nb exact pending updates) on genuine
    full-pivoting states: every W stays within the recursive bound sh_cert uses."""
    rng = np.random.default_rng(seed)
    m, n = 150, 130
    A = rng.random((m, n)) - 0.3
    if decay:
        A = A * np.exp(-decay * np.arange(n))[None, :]
    epochs = 3
    steps = nb * epochs + 1
    piv, X, Y, blocks = lu_states(A, steps + 1)
    pv = np.abs(np.array(piv))
    worst = 0.0
    stale0, rows_s, cols_s = blocks[0]
    s_cur = sh_scale(pv[0], mode)
    h = store((stale0 * s_cur).astype(np.float32), mode)  # pass 0 writes the shadow of A
    t0 = 0
    nok = 0
    for k in range(1, steps):
        PS = k - t0 + 1
        PE = k + 1  # no write-back inside the emulated exact epoch
        stale_k, rows_k, cols_k = blocks[k + 1]
        ri = [int(np.where(rows_s == q)[0][0]) for q in rows_k]
        ci = [int(np.where(cols_s == q)[0][0]) for q in cols_k]
        terms = []
        for q in range(t0, k + 1):
            xs = restrict(X[q], rows_k)
            ys = restrict(Y[q], cols_k) * s_cur
            xh, xl = split(-xs)
            yh, yl = split(ys)
            terms += [np.outer(xh, yh), np.outer(xh, yl), np.outer(xl, yh)]
        W = accumulate(h[np.ix_(ri, ci)], terms, mode, "seq")
        ea, ok = sh_cert(pv, k, PS, PE, nb, mode=mode)
        err = np.abs(W.astype(np.float64) / s_cur - stale_k).max()
        if ok:
            nok += 1
            worst = max(worst, err / ea)
        if PS == nb and k + 1 < steps:  # refresh: the new epoch's shadow from W (trailing block after k)
            s_new = sh_scale(2.0 * pv[k], mode)
            if ok:
                h = store((W * np.float32(s_new / s_cur)).astype(np.float32), mode)
            else:  # a refresh that cannot certify writes the exact values
                h = store((stale_k * s_new).astype(np.float32), mode)
            rows_s, cols_s, s_cur, t0 = rows_k, cols_k, s_new, k + 1
    assert nok > 0
    assert worst < 1.0, worst
    assert worst > 1e-3
