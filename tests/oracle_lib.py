"""ctypes binding of the CPU oracle (oracle/liboracle.so). TEST INFRASTRUCTURE ONLY.

Used by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg as the checker; the
product package never imports this module.
"""
import ctypes as C
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.path.join(ROOT, "oracle", "liboracle.so")

i64p = np.ctypeslib.ndpointer(dtype=np.int64, flags="C_CONTIGUOUS")
i32p = np.ctypeslib.ndpointer(dtype=np.int32, flags="C_CONTIGUOUS")
f64p = np.ctypeslib.ndpointer(dtype=np.float64, flags="C_CONTIGUOUS")


class OracleError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(msg)
        self.code = code


FAST_LIB_PATH = os.path.join(ROOT, "oracle", "liboracle_fast.so")
_libs = {}


def lib():
    return _bind(LIB_PATH)


def lib_fast():
    """The oracle's fast mode (tci_oracle.c "fast mode"; config 5 as stated): OpenMP rrLU (bitwise
    the same), CP evaluated factorised at the bond, site-tensor solves skipped (never read)."""
    return _bind(FAST_LIB_PATH)


def _bind(path):
    if path not in _libs:
        if not os.path.exists(path):
            import subprocess
            subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle")])
        L = C.CDLL(path)
        L.orc_last_error.restype = C.c_char_p
        L.orc_fill_uniform.argtypes = [f64p, C.c_int64, C.c_uint64, C.c_int64]
        L.orc_submatrixargmax.argtypes = [f64p, C.c_int64, C.c_int64, C.c_int64, i64p, C.c_int64,
                                          i64p, C.c_int64, C.c_int, C.POINTER(C.c_int64),
                                          C.POINTER(C.c_int64)]
        L.orc_rrlu_inplace.argtypes = [f64p, C.c_int64, C.c_int64, C.c_int64, C.c_int64, C.c_double,
                                       C.c_double, C.c_int, i64p, i64p, C.POINTER(C.c_int64),
                                       C.POINTER(C.c_double), C.c_int64]
        L.orc_rrlu.argtypes = [f64p, C.c_int64, C.c_int64, C.c_int64, C.c_double, C.c_double, C.c_int,
                               i64p, i64p, f64p, f64p, f64p, f64p, C.POINTER(C.c_int64),
                               C.POINTER(C.c_double), f64p]
        L.orc_batcheval.argtypes = [C.c_int, f64p, C.c_int64, i32p, C.c_int, i32p, C.c_int64, C.c_int,
                                    i32p, C.c_int64, C.c_int, C.c_int, f64p, C.POINTER(C.c_double)]
        L.orc_feval.argtypes = [C.c_int, f64p, C.c_int64, i32p, C.c_int, i32p]
        L.orc_feval.restype = C.c_double
        L.orc_sitetensor_solve.argtypes = [f64p, C.c_int64, f64p, C.c_int64, f64p]
        L.orc_div_shared_check.argtypes = [C.c_int64, C.c_uint64]
        L.orc_div_shared_check.restype = C.c_int64
        L.orc_convergencecriterion.argtypes = [i64p, f64p, i64p, C.c_int, C.c_double, C.c_int64,
                                               C.c_int, C.c_int]
        L.orc_tci_new.argtypes = [C.c_int, f64p, C.c_int64, i32p, C.c_int, i32p, C.c_int,
                                  C.POINTER(C.c_int)]
        L.orc_tci_new.restype = C.c_void_p
        L.orc_tci_free.argtypes = [C.c_void_p]
        L.orc_tci_updatepivots.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_double, C.c_double, C.c_int64]
        L.orc_tci_sweep2site.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_double, C.c_int64, C.c_int,
                                         C.c_int, C.c_int]
        L.orc_tci_sweep1site.argtypes = [C.c_void_p, C.c_int, C.c_double, C.c_double, C.c_int64, C.c_int]
        L.orc_tci_fillsitetensors.argtypes = [C.c_void_p]
        L.orc_tci_addglobalpivots.argtypes = [C.c_void_p, i32p, C.c_int]
        L.orc_tci_optimize.argtypes = [C.c_void_p, C.c_double, C.c_int64, C.c_int, C.c_int, C.c_int,
                                       C.c_int, C.c_int, C.c_int, i64p, f64p, C.POINTER(C.c_int)]
        L.orc_tci_L.argtypes = [C.c_void_p]
        L.orc_tci_maxsample.argtypes = [C.c_void_p]
        L.orc_tci_maxsample.restype = C.c_double
        for fn in ("orc_tci_iset_size", "orc_tci_jset_size", "orc_tci_sitetensor_size"):
            getattr(L, fn).argtypes = [C.c_void_p, C.c_int]
            getattr(L, fn).restype = C.c_int64
        L.orc_tci_iset_get.argtypes = [C.c_void_p, C.c_int, i32p]
        L.orc_tci_jset_get.argtypes = [C.c_void_p, C.c_int, i32p]
        L.orc_tci_pivoterrors.argtypes = [C.c_void_p, f64p, C.c_int64]
        L.orc_tci_pivoterrors.restype = C.c_int64
        L.orc_tci_bonderrors.argtypes = [C.c_void_p, f64p]
        L.orc_tci_sitetensor.argtypes = [C.c_void_p, C.c_int, f64p]
        L.orc_tci_evaluate.argtypes = [C.c_void_p, i32p, C.POINTER(C.c_double)]
        L.orc_rrlu_c128.argtypes = [f64p, C.c_int64, C.c_int64, C.c_int64, C.c_double, C.c_double,
                                    C.c_int, i64p, i64p, f64p, f64p, C.POINTER(C.c_int64),
                                    C.POINTER(C.c_double), f64p]
        L.orc_luci_c128.argtypes = [f64p, C.c_int64, C.c_int64, C.c_int64, C.c_double, C.c_double,
                                    C.c_int, i64p, i64p, f64p, f64p, f64p, C.POINTER(C.c_int64)]
        L.orc_cdiv.argtypes = [C.c_double] * 4 + [C.POINTER(C.c_double)] * 2
        L.orc_hypot.argtypes = [C.c_double, C.c_double]
        L.orc_hypot.restype = C.c_double
        L.orc_tci_save.argtypes = [C.c_void_p, C.c_char_p]
        L.orc_tci_load.argtypes = [C.c_void_p, C.c_char_p]
        _libs[path] = L
    return _libs[path]


def _check(st, L=None):
    if st != 0:
        raise OracleError(st, (L or lib()).orc_last_error().decode())


def fill_uniform(n, seed, offset=0):
    a = np.empty(n, dtype=np.float64)
    lib().orc_fill_uniform(a, n, seed, offset)
    return a


def submatrixargmax(A, rows, cols, f="abs2"):
    """0-based rows/cols lists -> (row, col), 0-based."""
    A = np.asfortranarray(A, dtype=np.float64)
    r = np.ascontiguousarray(rows, dtype=np.int64)
    c = np.ascontiguousarray(cols, dtype=np.int64)
    mr, mc = C.c_int64(), C.c_int64()
    flat = np.ascontiguousarray(A.ravel(order="F"))
    _check(lib().orc_submatrixargmax(flat, A.shape[0], A.shape[0], A.shape[1], r, len(r), c, len(c),
                                     1 if f == "abs2" else 0, C.byref(mr), C.byref(mc)))
    return mr.value, mc.value


def cdiv(z, w):
    """Julia's ComplexF64 `/` as restated in the oracle (Baudin-Smith robust division)."""
    re, im = C.c_double(), C.c_double()
    lib().orc_cdiv(z.real, z.imag, w.real, w.imag, C.byref(re), C.byref(im))
    return complex(re.value, im.value)


class OracleLUc:
    """rrlu(A::Matrix{ComplexF64}) restatement (matrixlu.jl:346-396 on complex entries)."""

    def __init__(self, A, maxrank=None, reltol=1e-14, abstol=0.0, leftorthogonal=True):
        A = np.asarray(A, dtype=np.complex128)
        m, n = A.shape
        maxrank = min(m, n) if maxrank is None else int(maxrank)
        mr = max(min(maxrank, m, n), 0)
        flat = np.ascontiguousarray(A.ravel(order="F")).view(np.float64)
        rp = np.zeros(max(m, 1), np.int64)
        cp = np.zeros(max(n, 1), np.int64)
        L = np.zeros(max(m * mr, 1), np.complex128)
        U = np.zeros(max(mr * n, 1), np.complex128)
        pe = np.zeros(mr + 1)
        npv, err = C.c_int64(), C.c_double()
        _check(lib().orc_rrlu_c128(flat, m, n, maxrank, reltol, abstol, int(leftorthogonal), rp, cp,
                                   L.view(np.float64), U.view(np.float64), C.byref(npv),
                                   C.byref(err), pe))
        k = npv.value
        self.m, self.n, self.npivot, self.error = m, n, k, err.value
        self.leftorthogonal = leftorthogonal
        self.rowpermutation = rp[:m].copy()
        self.colpermutation = cp[:n].copy()
        self.L = L[: m * k].reshape((m, k), order="F")
        self.U = U[: k * n].reshape((k, n), order="F")
        self.pivoterrors = pe[: k + 1].copy()


def luci_c128(A, maxrank=None, reltol=1e-14, abstol=0.0, leftorthogonal=True):
    """MatrixLUCI{ComplexF64} restatement -> (rowidx, colidx 0-based, pivoterrors, left, right)."""
    A = np.asarray(A, dtype=np.complex128)
    m, n = A.shape
    maxrank = min(m, n) if maxrank is None else int(maxrank)
    mr = max(min(maxrank, m, n), 0)
    flat = np.ascontiguousarray(A.ravel(order="F")).view(np.float64)
    ri = np.zeros(max(mr, 1), np.int64)
    ci = np.zeros(max(mr, 1), np.int64)
    pe = np.zeros(mr + 1)
    lf = np.zeros(max(m * mr, 1), np.complex128)
    rf = np.zeros(max(mr * n, 1), np.complex128)
    npv = C.c_int64()
    _check(lib().orc_luci_c128(flat, m, n, maxrank, reltol, abstol, int(leftorthogonal), ri, ci, pe,
                               lf.view(np.float64), rf.view(np.float64), C.byref(npv)))
    k = npv.value
    return (ri[:k].copy(), ci[:k].copy(), pe[: k + 1].copy(), lf[: m * k].reshape((m, k), order="F"),
            rf[: k * n].reshape((k, n), order="F"))


class OracleLU:
    """rrLU restatement result (matrixlu.jl:200-207) + MatrixLUCI factors (matrixluci.jl)."""

    def __init__(self, A, maxrank=None, reltol=1e-14, abstol=0.0, leftorthogonal=True):
        A = np.asarray(A, dtype=np.float64)
        m, n = A.shape
        maxrank = min(m, n) if maxrank is None else int(maxrank)
        mr = max(min(maxrank, m, n), 0)
        flat = np.ascontiguousarray(A.ravel(order="F"))
        rp = np.zeros(max(m, 1), np.int64)
        cp = np.zeros(max(n, 1), np.int64)
        L = np.zeros(max(m * mr, 1))
        U = np.zeros(max(mr * n, 1))
        left = np.zeros(max(m * mr, 1))
        right = np.zeros(max(mr * n, 1))
        pe = np.zeros(mr + 1)
        npv, err = C.c_int64(), C.c_double()
        _check(lib().orc_rrlu(flat, m, n, maxrank, reltol, abstol, int(leftorthogonal), rp, cp, L, U,
                              left, right, C.byref(npv), C.byref(err), pe))
        k = npv.value
        self.m, self.n, self.npivot, self.error = m, n, k, err.value
        self.leftorthogonal = leftorthogonal
        self.rowpermutation = rp[:m].copy()
        self.colpermutation = cp[:n].copy()
        self.L = L[: m * k].reshape((m, k), order="F")
        self.U = U[: k * n].reshape((k, n), order="F")
        self.left = left[: m * k].reshape((m, k), order="F")
        self.right = right[: k * n].reshape((k, n), order="F")
        self.pivoterrors = pe[: k + 1].copy()

    def rowindices(self):
        return self.rowpermutation[: self.npivot]

    def colindices(self):
        return self.colpermutation[: self.npivot]

    def left_lu(self):
        l = np.empty_like(self.L)
        l[self.rowpermutation, :] = self.L
        return l

    def right_lu(self):
        u = np.empty_like(self.U)
        u[:, self.colpermutation] = self.U
        return u


def rrlu_inplace_sample(A_flat, m, n, maxrank, pivot_limit, reltol=1e-14, abstol=0.0, leftorth=True):
    """Bounded CPU-baseline sample: runs `pivot_limit` pivots of _optimizerrlu! in place."""
    rp = np.zeros(m, np.int64)
    cp = np.zeros(n, np.int64)
    npv, err = C.c_int64(), C.c_double()
    _check(lib().orc_rrlu_inplace(A_flat, m, n, m, maxrank, reltol, abstol, int(leftorth), rp, cp,
                                  C.byref(npv), C.byref(err), pivot_limit))
    return npv.value, err.value, rp, cp


OMP_LIB_PATH = os.path.join(ROOT, "oracle", "libcpu_rrlu_omp.so")
_omp = {}


def omp_lib(path=None):
    """The all-core rrLU baseline (oracle/cpu_rrlu_omp.c); `path` selects a host-native build."""
    path = path or OMP_LIB_PATH
    if path not in _omp:
        if not os.path.exists(path):
            import subprocess
            subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle")])
        L = C.CDLL(path)
        L.cpu_rrlu_inplace_omp.argtypes = [f64p, C.c_int64, C.c_int64, C.c_int64, C.c_int64, C.c_double,
                                           C.c_double, C.c_int, i64p, i64p, C.POINTER(C.c_int64),
                                           C.POINTER(C.c_double), C.c_int64]
        L.cpu_rrlu_threads.restype = C.c_int
        _omp[path] = L
    return _omp[path]


def rrlu_inplace_omp(A_flat, m, n, maxrank, pivot_limit=-1, reltol=1e-14, abstol=0.0, leftorth=True,
                     path=None):
    """All-core baseline: same results as rrlu_inplace_sample, bitwise (cpu_rrlu_omp.c)."""
    rp = np.zeros(max(m, 1), np.int64)
    cp = np.zeros(max(n, 1), np.int64)
    npv, err = C.c_int64(), C.c_double()
    omp_lib(path).cpu_rrlu_inplace_omp(A_flat, m, n, m, maxrank, reltol, abstol, int(leftorth), rp, cp,
                                       C.byref(npv), C.byref(err), pivot_limit)
    return npv.value, err.value, rp, cp


def batcheval(kind, params, localdims, I, J, M):
    """I: (m, nl) int, J: (n, nr) int (1-based). Returns (out (m, prod(dc), n) F-order, maxabs)."""
    params = np.ascontiguousarray(params if params is not None and len(params) else [0.0], np.float64)
    ld = np.ascontiguousarray(localdims, np.int32)
    I = np.ascontiguousarray(np.asarray(I, np.int32).reshape(len(I), -1))
    J = np.ascontiguousarray(np.asarray(J, np.int32).reshape(len(J), -1))
    m, nl = I.shape
    n, nr = J.shape
    D = int(np.prod([localdims[nl + c] for c in range(M)])) if M else 1
    out = np.zeros(max(m * D * n, 1))
    mx = C.c_double(0.0)
    _check(lib().orc_batcheval(kind, params, len(params), ld, len(ld), I if I.size else np.zeros(1, np.int32),
                               m, nl, J if J.size else np.zeros(1, np.int32), n, nr, M, out, C.byref(mx)))
    return out[: m * D * n].reshape((m, D, n), order="F"), mx.value


def feval(kind, params, localdims, x):
    params = np.ascontiguousarray(params if params is not None and len(params) else [0.0], np.float64)
    return lib().orc_feval(kind, params, len(params), np.ascontiguousarray(localdims, np.int32),
                           len(localdims), np.ascontiguousarray(x, np.int32))


def sitetensor_solve(P, Pi1):
    P = np.asarray(P, np.float64)
    Pi1 = np.asarray(Pi1, np.float64)
    r = P.shape[0]
    R = Pi1.shape[0]
    T = np.zeros(R * r)
    _check(lib().orc_sitetensor_solve(np.ascontiguousarray(P.ravel(order="F")), r,
                                      np.ascontiguousarray(Pi1.ravel(order="F")), R, T))
    return T.reshape((R, r), order="F")


def convergencecriterion(ranks, errors, ngp, tol, maxbonddim, ncheck, checkconvglobalpivot=True):
    return bool(lib().orc_convergencecriterion(np.ascontiguousarray(ranks, np.int64),
                                               np.ascontiguousarray(errors, np.float64),
                                               np.ascontiguousarray(ngp, np.int64), len(ranks), tol,
                                               maxbonddim, ncheck, int(checkconvglobalpivot)))


INT64_MAX = np.iinfo(np.int64).max


class OracleTCI2:
    """CPU restatement of TensorCI2 (tensorci2.jl:50-137) in deterministic mode."""

    def __init__(self, kind, params, localdims, initialpivots=None, fast=False):
        self._L = lib_fast() if fast else lib()
        self.localdims = [int(d) for d in localdims]
        L = len(self.localdims)
        if initialpivots is None:
            initialpivots = [[1] * L]
        piv = np.ascontiguousarray(np.asarray(initialpivots, np.int32).reshape(-1, L))
        params = np.ascontiguousarray(params if params is not None and len(params) else [0.0], np.float64)
        st = C.c_int(0)
        self._h = self._L.orc_tci_new(kind, params, len(params), np.ascontiguousarray(self.localdims, np.int32),
                                    L, piv, piv.shape[0], C.byref(st))
        _check(st.value, self._L)

    def _chk(self, st):
        _check(st, self._L)

    def save(self, path):
        """Checkpoint (orc_tci_save): sets, history entry, errors, maxsample."""
        self._chk(self._L.orc_tci_save(self._h, path.encode()))

    def load(self, path):
        self._chk(self._L.orc_tci_load(self._h, path.encode()))

    def __del__(self):
        if getattr(self, "_h", None):
            self._L.orc_tci_free(self._h)
            self._h = None

    @property
    def L(self):
        return len(self.localdims)

    def updatepivots(self, b, leftorthogonal=True, reltol=1e-14, abstol=0.0, maxbonddim=INT64_MAX):
        self._chk(self._L.orc_tci_updatepivots(self._h, b, int(leftorthogonal), reltol, abstol, maxbonddim))

    def sweep1site(self, forward=True, reltol=1e-14, abstol=0.0, maxbonddim=INT64_MAX, updatetensors=True):
        self._chk(self._L.orc_tci_sweep1site(self._h, int(forward), reltol, abstol, maxbonddim, int(updatetensors)))

    def sweep2site(self, niter=2, abstol=1e-8, maxbonddim=INT64_MAX, sweepstrategy="backandforth",
                   strictlynested=False, fillsitetensors=True, iter1=1):
        """iter1: the number of the first half-sweep (odd = forward under :backandforth), so a
        sweep2site! call can be split into half-sweeps with identical results."""
        self._chk(self._L.orc_tci_sweep2site(self._h, niter, iter1, abstol, maxbonddim,
                                        0 if sweepstrategy == "backandforth" else 1, int(strictlynested),
                                        int(fillsitetensors)))

    def addglobalpivots(self, pivots):
        piv = np.ascontiguousarray(np.asarray(pivots, np.int32).reshape(-1, self.L))
        self._chk(self._L.orc_tci_addglobalpivots(self._h, piv, piv.shape[0]))

    def makecanonical(self, reltol=1e-14, abstol=0.0, maxbonddim=INT64_MAX):
        self.sweep1site(True, 0.0, 0.0, INT64_MAX, False)
        self.sweep1site(False, reltol, abstol, maxbonddim, False)
        self.sweep1site(True, reltol, abstol, maxbonddim, True)

    def optimize(self, tolerance=1e-8, maxbonddim=INT64_MAX, maxiter=20, sweepstrategy="backandforth",
                 normalizeerror=True, ncheckhistory=3, strictlynested=False, checkconvglobalpivot=True):
        ranks = np.zeros(maxiter, np.int64)
        errors = np.zeros(maxiter)
        nit = C.c_int(0)
        self._chk(self._L.orc_tci_optimize(self._h, tolerance, maxbonddim, maxiter,
                                      0 if sweepstrategy == "backandforth" else 1, int(normalizeerror),
                                      ncheckhistory, int(strictlynested), int(checkconvglobalpivot), ranks,
                                      errors, C.byref(nit)))
        k = nit.value
        return ranks[:k].tolist(), errors[:k].tolist()

    def Iset(self, p):
        n = self._L.orc_tci_iset_size(self._h, p)
        out = np.zeros(max(n * p, 1), np.int32)
        self._L.orc_tci_iset_get(self._h, p, out)
        return out[: n * p].reshape(n, p)

    def Jset(self, p):
        n = self._L.orc_tci_jset_size(self._h, p)
        w = self.L - 1 - p
        out = np.zeros(max(n * w, 1), np.int32)
        self._L.orc_tci_jset_get(self._h, p, out)
        return out[: n * w].reshape(n, w)

    def linkdims(self):
        return [int(self._L.orc_tci_iset_size(self._h, p + 1)) for p in range(self.L - 1)]

    def rank(self):
        return max(self.linkdims())

    @property
    def maxsamplevalue(self):
        return self._L.orc_tci_maxsample(self._h)

    @property
    def pivoterrors(self):
        out = np.zeros(1 << 16)
        n = self._L.orc_tci_pivoterrors(self._h, out, len(out))
        return out[:n].copy()

    @property
    def bonderrors(self):
        out = np.zeros(self.L - 1)
        self._L.orc_tci_bonderrors(self._h, out)
        return out

    def pivoterror(self):
        return float(np.max(self.bonderrors))

    def sitetensor(self, p):
        n = self._L.orc_tci_sitetensor_size(self._h, p)
        out = np.zeros(max(n, 1))
        self._L.orc_tci_sitetensor(self._h, p, out)
        a = self._L.orc_tci_iset_size(self._h, p)
        b = self._L.orc_tci_jset_size(self._h, p)
        return out[:n].reshape((a, self.localdims[p], b), order="F")

    def evaluate(self, idx):
        v = C.c_double()
        self._chk(self._L.orc_tci_evaluate(self._h, np.ascontiguousarray(idx, np.int32), C.byref(v)))
        return v.value


def crossinterpolate2(kind, params, localdims, initialpivots=None, fast=False, **kw):
    t = OracleTCI2(kind, params, localdims, initialpivots, fast=fast)
    ranks, errors = t.optimize(**kw)
    return t, ranks, errors
