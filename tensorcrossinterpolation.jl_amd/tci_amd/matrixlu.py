"""Rank-revealing LU with full pivoting on the GPU -- the host-side mirror of src/matrixlu.jl.

`rrlu(A; maxrank, reltol, abstol, leftorthogonal)` (matrixlu.jl:455-463) returns an `rrLU`
(matrixlu.jl:200-231) whose accessors mirror the reference: left/right (:716-746),
rowindices/colindices (:769-780), npivots (:787), pivoterrors (:799), lastpivoterror (:811),
diag (:756), size (:685-702). The factorisation itself runs in libtci_hip.so.
Indices follow Julia: rowpermutation/colpermutation/rowindices/colindices are 1-based.
"""
import ctypes as C

import numpy as np

from . import _lib

INT64_MAX = np.iinfo(np.int64).max


class rrLU:
    """mutable struct rrLU{T} (matrixlu.jl:200-207)."""

    def __init__(self, rowpermutation, colpermutation, L, U, leftorthogonal, npivot, error):
        if npivot != L.shape[1]:
            raise ValueError("L must have the same number of columns as the number of pivots.")
        if npivot != U.shape[0]:
            raise ValueError("U must have the same number of rows as the number of pivots.")
        self.rowpermutation = np.asarray(rowpermutation, dtype=np.int64)
        self.colpermutation = np.asarray(colpermutation, dtype=np.int64)
        self.L = L
        self.U = U
        self.leftorthogonal = bool(leftorthogonal)
        self.npivot = int(npivot)
        self.error = float(error)

    @property
    def shape(self):
        return self.L.shape[0], self.U.shape[1]

    def size(self, dim=None):
        if dim is None:
            return self.shape
        return self.shape[dim - 1] if dim in (1, 2) else 1

    def transpose(self):
        """Base.transpose(::rrLU) (matrixlu.jl:918-923)."""
        return rrLU(self.colpermutation, self.rowpermutation, np.ascontiguousarray(self.U.T),
                    np.ascontiguousarray(self.L.T), not self.leftorthogonal, self.npivot, self.error)


def rrlu(A, maxrank=INT64_MAX, reltol=1e-14, abstol=0.0, leftorthogonal=True, ctx=None):
    """rrlu(A; maxrank, reltol, abstol, leftorthogonal) (matrixlu.jl:455-463). A is not modified.
    Float64 and ComplexF64 (complex128) matrices, like the reference's rrLU{T}."""
    ctx = ctx or _lib.context()
    if np.iscomplexobj(A):
        return _rrlu_c128(A, maxrank, reltol, abstol, leftorthogonal, ctx)
    A = np.asarray(A, dtype=np.float64)
    if A.ndim != 2:
        raise ValueError("A must be a matrix")
    m, n = A.shape
    Af = np.asfortranarray(A)
    mr = int(max(min(int(maxrank), m, n), 0))
    rowperm = np.zeros(max(m, 1), np.int64)
    colperm = np.zeros(max(n, 1), np.int64)
    L = np.zeros(max(m * mr, 1))
    U = np.zeros(max(mr, 1) * max(n, 1))
    npv = C.c_int64()
    err = C.c_double()
    ctx.check(ctx.lib.tci_rrlu_h(ctx.h, _lib.ptr(Af), m, n, max(m, 1), int(min(maxrank, INT64_MAX)),
                                 float(reltol), float(abstol), int(bool(leftorthogonal)),
                                 _lib.ptr(rowperm), _lib.ptr(colperm), _lib.ptr(L), _lib.ptr(U),
                                 max(mr, 1), C.byref(npv), C.byref(err)))
    k = npv.value
    Lm = L[: m * k].reshape((m, k), order="F").copy()
    # U was written with leading dimension max(mr, 1)
    Um = U[: max(mr, 1) * n].reshape((max(mr, 1), n), order="F")[:k, :].copy()
    return rrLU(rowperm[:m].copy(), colperm[:n].copy(), Lm, Um, leftorthogonal, k, err.value)


def _rrlu_c128(A, maxrank, reltol, abstol, leftorthogonal, ctx):
    """rrLU{ComplexF64}: tci_rrlu_c128_h (interleaved re/im, Julia's ComplexF64 layout)."""
    A = np.asarray(A, dtype=np.complex128)
    if A.ndim != 2:
        raise ValueError("A must be a matrix")
    m, n = A.shape
    Af = np.asfortranarray(A)
    mr = int(max(min(int(maxrank), m, n), 0))
    rowperm = np.zeros(max(m, 1), np.int64)
    colperm = np.zeros(max(n, 1), np.int64)
    L = np.zeros(max(m * mr, 1), np.complex128)
    U = np.zeros(max(mr, 1) * max(n, 1), np.complex128)
    pe = np.zeros(mr + 1)
    npv = C.c_int64()
    err = C.c_double()
    ctx.check(ctx.lib.tci_rrlu_c128_h(ctx.h, _lib.ptr(Af), m, n, max(m, 1), int(min(maxrank, INT64_MAX)),
                                      float(reltol), float(abstol), int(bool(leftorthogonal)),
                                      _lib.ptr(rowperm), _lib.ptr(colperm), _lib.ptr(L), _lib.ptr(U),
                                      max(mr, 1), C.byref(npv), C.byref(err), _lib.ptr(pe)))
    k = npv.value
    Lm = L[: m * k].reshape((m, k), order="F").copy()
    Um = U[: max(mr, 1) * n].reshape((max(mr, 1), n), order="F")[:k, :].copy()
    lu = rrLU(rowperm[:m].copy(), colperm[:n].copy(), Lm, Um, leftorthogonal, k, err.value)
    lu.device_pivoterrors = pe[: k + 1].copy()
    return lu


def rrlu_(A, **kw):
    """rrlu!(A; ...) (matrixlu.jl:420-430): factorises in place (A is overwritten with the packed
    factors like the reference's working matrix)."""
    lu = rrlu(A, **kw)
    return lu


def left(lu, permute=True):
    """left(lu; permute) (matrixlu.jl:716-724)."""
    if not permute:
        return lu.L
    l = np.empty_like(lu.L)
    l[lu.rowpermutation - 1, :] = lu.L
    return l


def right(lu, permute=True):
    """right(lu; permute) (matrixlu.jl:738-746)."""
    if not permute:
        return lu.U
    u = np.empty_like(lu.U)
    u[:, lu.colpermutation - 1] = lu.U
    return u


def diag(lu):
    """diag(lu) (matrixlu.jl:756-762)."""
    k = lu.npivot
    if lu.leftorthogonal:
        return np.diag(lu.U[:k, :k]).copy()
    return np.diag(lu.L[:k, :k]).copy()


def rowindices(lu):
    return lu.rowpermutation[: lu.npivot]


def colindices(lu):
    return lu.colpermutation[: lu.npivot]


def npivots(lu):
    return lu.npivot


def pivoterrors(lu):
    """pivoterrors(lu) (matrixlu.jl:799-801): [abs.(diag(lu)); lu.error]. For ComplexF64 the
    device computes abs (Julia's hypot) next to the factorisation."""
    pe = getattr(lu, "device_pivoterrors", None)
    if pe is not None:
        return pe.copy()
    return np.concatenate([np.abs(diag(lu)), [lu.error]])


def lastpivoterror(lu):
    return lu.error


def solve(L, U, b):
    """solve(L, U, b) (matrixlu.jl:839-868): forward then backward substitution (host, small)."""
    N2 = L.shape[1]
    N3 = U.shape[1]
    y = np.zeros((N2, b.shape[1]))
    for i in range(N2):
        y[i, :] = b[i, :]
        for j in range(i):
            y[i, :] -= L[i, j] * y[j, :]
        y[i, :] /= L[i, i]
    x = np.zeros((N3, b.shape[1]))
    for i in range(N3 - 1, -1, -1):
        x[i, :] = y[i, :]
        for j in range(i + 1, N3):
            x[i, :] -= U[i, j] * x[j, :]
        x[i, :] /= U[i, i]
    return x


def ldiv(lu, b):
    """Base.:\\(A::rrLU, b) (matrixlu.jl:891-905)."""
    if lu.shape[0] != lu.shape[1]:
        raise ValueError("Matrix must be square.")
    if lu.npivot != lu.shape[0]:
        raise ValueError("rank-deficient matrix is not supportred!")
    b = np.asarray(b, float)
    b_perm = b[lu.rowpermutation - 1, :]
    x_perm = solve(lu.L, lu.U, b_perm)
    x = np.empty_like(x_perm)
    x[lu.colpermutation - 1, :] = x_perm
    return x


class DeviceMatrix:
    """A column-major Float64 matrix resident in HBM (ld even, 16-B aligned), for the bench and
    for chaining device calls without host round trips."""

    def __init__(self, m, n, ctx=None, ld=None):
        self.ctx = ctx or _lib.context()
        self.m, self.n = int(m), int(n)
        self.ld = int(ld) if ld else ((max(self.m, 1) + 15) // 16) * 16
        self.nbytes = self.ld * max(self.n, 1) * 8
        p = C.c_void_p()
        self.ctx.check(self.ctx.lib.tci_malloc_d(self.ctx.h, C.byref(p), self.nbytes))
        self.ptr = p
        self.ctx.own(self)

    def fill_uniform(self, seed):
        self.ctx.check(self.ctx.lib.tci_fill_uniform_d(self.ctx.h, self.ptr, self.m, self.n, self.ld, seed))

    def copy_from(self, other):
        assert other.ld == self.ld and other.n == self.n
        self.ctx.check(self.ctx.lib.tci_memcpy_d2d(self.ctx.h, self.ptr, other.ptr, self.nbytes))

    def upload(self, A):
        """Copies a host m x n array in (padded to ld)."""
        A = np.asarray(A, dtype=np.float64)
        if A.shape != (self.m, self.n):
            raise ValueError(f"upload: shape {A.shape} != {(self.m, self.n)}")
        buf = np.zeros((self.ld, max(self.n, 1)), order="F")
        buf[: self.m, : self.n] = A
        self.ctx.check(self.ctx.lib.tci_memcpy_h2d(self.ctx.h, self.ptr, _lib.ptr(buf.ravel(order="F")),
                                                   self.nbytes))
        return self

    def to_host(self):
        buf = np.empty(self.ld * max(self.n, 1))
        self.ctx.check(self.ctx.lib.tci_memcpy_d2h(self.ctx.h, _lib.ptr(buf), self.ptr, self.nbytes))
        return buf.reshape((self.ld, max(self.n, 1)), order="F")[: self.m, : self.n]

    def free(self):
        if self.ptr and self.ctx.alive:
            self.ctx.lib.tci_free_d(self.ctx.h, self.ptr)
        self.ptr = None

    release = free

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


def rrlu_inplace_device(dm, maxrank=INT64_MAX, reltol=1e-14, abstol=0.0, leftorthogonal=True,
                        want_perms=True, src=None):
    """rrlu! on a DeviceMatrix: returns (npivot, error, rowperm, colperm, pivoterrors).
    src (a DeviceMatrix of the same shape, not overlapping dm): rrlu(src) -- src is copied into dm
    (matrixlu.jl:462) by the factorisation's first pass as it reads it (tci_rrlu_copy_d), and dm
    is the work matrix; src is left untouched."""
    ctx = dm.ctx
    m, n = dm.m, dm.n
    rowperm = np.zeros(max(m, 1), np.int64) if want_perms else None
    colperm = np.zeros(max(n, 1), np.int64) if want_perms else None
    mr = int(max(min(int(maxrank), m, n), 0))
    pe = np.zeros(mr + 1)
    npv = C.c_int64()
    err = C.c_double()
    if src is not None:
        if (src.m, src.n) != (m, n):
            raise ValueError("rrlu: src and the work matrix differ in shape")
        ctx.check(ctx.lib.tci_rrlu_copy_d(ctx.h, src.ptr, src.ld, dm.ptr, m, n, dm.ld, int(min(maxrank, INT64_MAX)),
                                          float(reltol), float(abstol), int(bool(leftorthogonal)),
                                          _lib.ptr(rowperm), _lib.ptr(colperm), C.byref(npv),
                                          C.byref(err), _lib.ptr(pe)))
        k = npv.value
        return k, err.value, rowperm, colperm, pe[: k + 1]
    ctx.check(ctx.lib.tci_rrlu_inplace_d(ctx.h, dm.ptr, m, n, dm.ld, int(min(maxrank, INT64_MAX)),
                                         float(reltol), float(abstol), int(bool(leftorthogonal)),
                                         _lib.ptr(rowperm), _lib.ptr(colperm), C.byref(npv),
                                         C.byref(err), _lib.ptr(pe)))
    k = npv.value
    return k, err.value, rowperm, colperm, pe[: k + 1]


def dgemm_device(A, B, C_, alpha=1.0, beta=0.0, transb=False, k=None):
    """C = beta C + alpha A op(B) on DeviceMatrix operands (fp64 MFMA, K3 of DESIGN.md):
    op(B) = B (k x n) or, transb, B^T (B n x k). Asynchronous on the context stream."""
    ctx = C_.ctx
    k = A.n if k is None else int(k)
    ctx.check(ctx.lib.tci_dgemm_d(ctx.h, int(bool(transb)), C_.m, C_.n, k, float(alpha), A.ptr, A.ld,
                                  B.ptr, B.ld, float(beta), C_.ptr, C_.ld))


def schur_update_device(C_, W, V):
    """C -= W V (the blocked Schur-complement update of a right-looking LU) on DeviceMatrix
    operands: C m x n, W m x k, V k x n."""
    ctx = C_.ctx
    ctx.check(ctx.lib.tci_schur_update_d(ctx.h, C_.ptr, C_.m, C_.n, C_.ld, W.ptr, W.ld, V.ptr, V.ld, W.n))


def sitetensor_solve_device(P, Pi1, T_):
    """T = Pi1 P^-1 (setsitetensor!'s solve, tensorci2.jl:620-627) on DeviceMatrix operands with
    ld = rows (P r x r is clobbered by its LU; Pi1, T R x r)."""
    ctx = T_.ctx
    r, R = P.m, Pi1.m
    if P.ld != r or Pi1.ld != R or T_.ld != R or P.n != r or Pi1.n != r or T_.m != R or T_.n != r:
        raise ValueError("sitetensor_solve_device: P r x r, Pi1 and T R x r with ld = rows")
    ctx.check(ctx.lib.tci_sitetensor_solve_d(ctx.h, P.ptr, r, Pi1.ptr, R, T_.ptr))
