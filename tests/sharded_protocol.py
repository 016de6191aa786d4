"""Test infrastructure: a numpy restatement of the column-sharded rrLU PROTOCOL of
tci_rrlu_sharded_d (include/tci_hip.h), for the CPU (gloo) tests.

Each rank holds the columns [c0, c0 + nloc) of the matrix. Per pivot k it finds the argmax of
abs2 over ITS part of the trailing block in the reference's scan order (submatrixargmax,
/root/reference/src/matrixlu.jl:46-87: column position, then row position, strict '>'), sends the
candidate (abs2, value, column position, row position, global column, row) to every rank
(all-gather); every rank reduces the candidates to the same winner, the rank owning the winning
column contributes that column's current values and the others zeros, and an element-wise max of
the contributions as uint64 bit patterns gives every rank the column (candidate first: 8 m bytes
per pivot, not N x 8 m); then every rank commits the same winner: stop test of _optimizerrlu!
(matrixlu.jl:359-368), swaprow!/swapcol! as position maps, normalisation and the rank-1 update of
addpivot! (matrixlu.jl:295-322, separate multiply and subtract) on its own columns, with the pivot
column taken from the winner's record. The result must equal the unsharded oracle bit for bit --
which checks the protocol (tie order across ranks, the stop test, the replicated maps), not the
device kernels (those are checked against the same oracle in tests/test_gpu_sharded.py).

fused=True is the one-collective form (tci_set_shard_exchange mode 2, k_shard_pack): every rank
all-gathers its candidate TOGETHER with its own candidate column (bits), and every rank takes the
winning column from the winner's slot -- the same winner, the same bits, one exchange per pivot.
"""
import numpy as np


def sharded_rrlu(A_loc, m, n, c0, allgather, allreduce_max_u64, maxrank=None, reltol=1e-14, abstol=0.0,
                 leftorth=True, fused=False):
    """A_loc: this rank's m x nloc block (physical = original indices). allgather(vec) returns the
    rank-major concatenation of every rank's equal-length float64 vector; allreduce_max_u64(words)
    the element-wise max over the ranks of uint64 vectors. Returns npivot, error, rowperm, colperm
    (0-based), L (m x np), this rank's U columns (np x n, zeros elsewhere)."""
    A = np.array(A_loc, dtype=np.float64, order="F")
    nloc = A.shape[1]
    mr = min(m, n) if maxrank is None else min(int(maxrank), m, n)
    rowpos = np.arange(m)
    rowphys = np.arange(m)
    colpos = np.arange(n)
    colphys = np.arange(n)
    Lcols, Urows, piv = [], [], []
    maxerror, error, npv = 0.0, np.nan, 0
    for k in range(mr):
        # local argmax over trailing rows / local trailing columns, reference scan order
        best = (-1.0, 0.0, 2 ** 31 - 1, 2 ** 31 - 1, -1, -1)
        R = np.where(rowpos >= k)[0]
        Cc = np.array([jl for jl in range(nloc) if colpos[c0 + jl] >= k], dtype=np.int64)
        if len(R) and len(Cc):
            sub = A[np.ix_(R, Cc)]
            a2 = sub * sub
            mx = a2.max()
            ii, jj = np.nonzero(a2 == mx)
            # ties: smallest column position, then smallest row position
            key = [(colpos[c0 + Cc[j]], rowpos[R[i]], i, j) for i, j in zip(ii, jj)]
            _, _, i, j = min(key)
            best = (float(mx), float(sub[i, j]), int(colpos[c0 + Cc[j]]), int(rowpos[R[i]]), int(c0 + Cc[j]),
                    int(R[i]))
        if fused:  # [candidate | own candidate column as bits], one all-gather
            own = A[:, best[4] - c0].copy() if best[4] >= 0 else np.zeros(m)
            allr = allgather(np.concatenate([np.array(best, np.float64), own])).reshape(-1, 6 + m)
        else:
            allr = allgather(np.array(best, np.float64)).reshape(-1, 6)
        win, wr = None, -1
        for r in range(allr.shape[0]):
            c = tuple(allr[r, :6])
            c = (c[0], c[1], int(c[2]), int(c[3]), int(c[4]), int(c[5]))
            if c[4] >= 0 and (win is None or _better(c, win)):
                win, wr = c, r
        a2, val, cp, rp, pc, pr = win
        if fused:
            col = np.ascontiguousarray(allr[wr, 6:]).view(np.uint64).view(np.float64)
        else:
            # the owner of the winning column contributes it (as bits), the others zeros
            mine = c0 <= pc < c0 + nloc
            contrib = A[:, pc - c0].copy().view(np.uint64) if mine else np.zeros(m, np.uint64)
            col = np.ascontiguousarray(allreduce_max_u64(contrib), np.uint64).view(np.float64)
        err = abs(val)
        error = err
        if (err < reltol * maxerror or err < abstol) and k > 0:
            break
        maxerror = max(maxerror, err)
        # swaprow!(k, rp), swapcol!(k, cp)
        rk, ck = rowphys[k], colphys[k]
        rowphys[k], rowphys[rp] = pr, rk
        rowpos[pr], rowpos[rk] = k, rp
        colphys[k], colphys[cp] = pc, ck
        colpos[pc], colpos[ck] = k, cp
        trail_r = rowpos > k
        trail_c = np.array([colpos[c0 + j] > k for j in range(nloc)], bool)
        x = col.copy()
        if leftorth:
            x[trail_r] = x[trail_r] / val
        y = A[pr, :].copy()
        if not leftorth:
            y[trail_c] = y[trail_c] / val
        Lcols.append(x)
        Urows.append(y)
        piv.append(val)
        # rank-1 update of the local trailing block: A -= x * y (separate multiply and subtract)
        R = np.where(trail_r)[0]
        Cc = np.where(trail_c)[0]
        if len(R) and len(Cc):
            A[np.ix_(R, Cc)] = A[np.ix_(R, Cc)] - np.multiply.outer(x[R], y[Cc])
        npv = k + 1
    if npv >= min(m, n):
        error = 0.0
    # position-order factors (rrLU accessors, matrixlu.jl:685-813)
    L = np.zeros((m, npv))
    U = np.zeros((npv, n))
    for t in range(npv):
        for pos in range(m):
            if pos < t:
                continue
            L[pos, t] = (1.0 if leftorth else piv[t]) if pos == t else Lcols[t][rowphys[pos]]
        for pos in range(n):
            pcol = colphys[pos] - c0
            if pos < t or not (0 <= pcol < nloc):
                continue
            U[t, pos] = (piv[t] if leftorth else 1.0) if pos == t else Urows[t][pcol]
    return npv, error, rowphys.copy(), colphys.copy(), L, U


def _better(a, b):
    """(abs2, value, column position, row position, ...): larger abs2, then smaller column
    position, then smaller row position."""
    return a[0] > b[0] or (a[0] == b[0] and (a[2] < b[2] or (a[2] == b[2] and a[3] < b[3])))
