"""HostFunctionEvaluator -- the user's own `f` (or BatchEvaluator) on the device rrLU path.

The reference's main use is an arbitrary closure, evaluated point by point by the generic
`_batchevaluate_dispatch` (batcheval.jl:131-175), or a user `BatchEvaluator` reached through its
batch method (batcheval.jl:196-214), e.g. `ThreadedBatchEvaluator` (:247-308) -- the contract is
docs/src/index.md:174-243. A device kernel cannot run that code, so here the batch is evaluated on
the host by a callback the library invokes (tci_func_create_host, include/tci_hip.h): the Pi block
of a 2-site update is filled on the host ONCE, uploaded into HBM, and everything after it --
max|Pi|, the rrLU, the MatrixLUCI factors, the site-tensor solve, the device memo -- runs on the GPU,
through exactly the same entries as the catalog integrands (tci_update_pivots_h, tci_sitetensor_h,
the native sweep driver tci_tci2_sweep2site).

Three ways to give f:
  * pointwise (default): f(x) with x a list of 1-based ints -> float. threads > 1 spreads the
    points over a thread pool, the analogue of ThreadedBatchEvaluator (pays off when f releases
    the GIL, e.g. numpy-heavy f);
  * vectorized=True: f(X) with X an (N, L) int32 array of points -> N values (one call per batch);
  * batch=True: f(I, J, M) with I (m, nl), J (n, nr) int32 arrays -> array of shape
    (m, d_{nl+1..nl+M}..., n) -- a user BatchEvaluator's (f)(Iset, Jset, Val(M)).
Single points f(x) (TensorCI2 construction, the global pivot search's scalar calls,
globalpivotfinder.jl:236) are evaluated on the host directly, as the reference calls obj.f.
"""
import ctypes as C

import numpy as np

from . import _lib

# int (*)(void* user, const int32* I, int64 m, int32 nl, const int32* J, int64 n, int32 nr,
#         int32 M, double* out, int64 ldo)
HOST_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.POINTER(C.c_int32), C.c_int64, C.c_int32,
                      C.POINTER(C.c_int32), C.c_int64, C.c_int32, C.c_int32, C.POINTER(C.c_double),
                      C.c_int64)


def _table(p, count, width):
    if count * width == 0:
        return np.zeros((count, width), np.int32)
    return np.ctypeslib.as_array(p, shape=(count * width,)).reshape(count, width).copy()


class HostFunctionEvaluator:
    """BatchEvaluator{Float64} over a host function; the factorisation path is the device's."""

    kind = 10  # TCI_F_HOST

    def __init__(self, f, localdims, ctx=None, threads=1, vectorized=False, batch=False, name=None):
        if vectorized and batch:
            raise ValueError("choose one of vectorized / batch")
        self.f = f
        self.localdims = [int(d) for d in localdims]
        self.L = len(self.localdims)
        self.ctx = ctx or _lib.context()
        self.threads = max(1, int(threads))
        self.vectorized = bool(vectorized)
        self.is_batch = bool(batch)
        self.name = name or getattr(f, "__name__", "host_f")
        self.nbatches = 0   # batches the library asked for
        self.npoints = 0    # points evaluated on the host through the callback
        self.host_seconds = 0.0
        self._pool = None
        self._cb = HOST_FN(self._callback)  # kept alive as long as the tci_func
        h = C.c_void_p()
        self.ctx.check(self.ctx.lib.tci_func_create_host(self.ctx.h, self._cb, None,
                                                         np.ascontiguousarray(self.localdims, np.int32),
                                                         self.L, C.byref(h)))
        self.h = h
        self.ctx.own(self)

    def release(self):
        if getattr(self, "h", None) and self.ctx.alive:
            self.ctx.lib.tci_func_destroy(self.h)
        self.h = None
        if self._pool is not None:
            self._pool.shutdown(wait=False)
            self._pool = None

    def __del__(self):
        try:
            self.release()
        except Exception:
            pass

    # -- host evaluation -------------------------------------------------------------------
    def _points_host(self, X):
        """f at every row of X (N x L, 1-based) in row order."""
        X = np.ascontiguousarray(X, np.int32)
        N = len(X)
        if N == 0:
            return np.zeros(0)
        if self.vectorized:
            v = np.asarray(self.f(X), np.float64).reshape(-1)
            if v.size != N:
                raise ValueError(f"vectorized f returned {v.size} values for {N} points")
            return v
        if self.is_batch:  # a batch evaluator asked for single points: I = the points, J = {()}
            v = np.asarray(self.f(X, np.zeros((1, 0), np.int32), 0), np.float64)
            return v.reshape(-1)
        out = np.empty(N)
        f = self.f
        if self.threads == 1 or N < 4 * self.threads:
            for t, x in enumerate(X.tolist()):
                out[t] = f(x)
            return out
        if self._pool is None:
            from concurrent.futures import ThreadPoolExecutor
            self._pool = ThreadPoolExecutor(self.threads)
        rows = X.tolist()
        bounds = np.linspace(0, N, self.threads + 1).astype(int)

        def work(a, b):
            for t in range(a, b):
                out[t] = f(rows[t])

        list(self._pool.map(lambda ab: work(*ab), zip(bounds[:-1], bounds[1:])))
        return out

    def _batch_host(self, I, J, M):
        """(m * D) x n column-major values of f over I x (centre) x J (batcheval.jl:157-171)."""
        m, nl = I.shape
        n, nr = J.shape
        if nl + M + nr != self.L or M not in (0, 1):
            raise ValueError("Invalid number of central indices")
        D = self.localdims[nl] if M == 1 else 1
        if self.is_batch:
            v = np.asarray(self.f(I, J, M), np.float64)
            if v.size != m * D * n:
                raise ValueError(f"batch evaluator returned {v.shape}, expected {(m,) + (D,) * M + (n,)}")
            return v.reshape((m * D, n), order="F")
        # points ordered i fastest, then c, then j: P[j, c, i] = [I_i..., c, J_j...]
        P = np.empty((n, D, m, self.L), np.int32)
        P[..., :nl] = I[None, None, :, :]
        if M == 1:
            P[..., nl] = (np.arange(D, dtype=np.int32) + 1)[None, :, None]
        P[..., nl + M:] = J[:, None, None, :]
        return self._points_host(P.reshape(-1, self.L)).reshape((m * D, n), order="F")

    def _callback(self, _user, pI, m, nl, pJ, n, nr, M, pout, ldo):
        import time
        try:
            t0 = time.perf_counter()
            I = _table(pI, m, nl)
            J = _table(pJ, n, nr)
            vals = self._batch_host(I, J, M)
            mR = vals.shape[0]
            out = np.ctypeslib.as_array(pout, shape=(n * ldo,)).reshape(n, ldo)
            out[:, :mR] = vals.T
            self.nbatches += 1
            self.npoints += vals.size
            self.host_seconds += time.perf_counter() - t0
            return 0
        except BaseException as e:  # re-raised by Context.check on TCI_ERR_HOST
            _lib.set_host_exception(e)
            return 1

    # -- BatchEvaluator interface ------------------------------------------------------------
    def __call__(self, x, Jset=None, M=None):
        if Jset is not None:
            return self.batch(x, Jset, M)
        if self.is_batch:
            return float(self._points_host(np.asarray(x, np.int32).reshape(1, self.L))[0])
        return float(self.f([int(v) for v in x]) if not self.vectorized
                     else self._points_host(np.asarray(x, np.int32).reshape(1, self.L))[0])

    def points(self, X):
        """f at each row of X (host; the reference's scalar f(x) calls)."""
        return self._points_host(np.asarray(X, np.int32).reshape(-1, self.L))

    def pi(self, I, J, M=0):
        """(|I| * D) x |J| Fortran matrix and max|.| (Julia's NaN-propagating max, util.jl:34)."""
        I = np.ascontiguousarray(np.asarray(I, np.int32))
        J = np.ascontiguousarray(np.asarray(J, np.int32))
        vals = self._batch_host(I, J, int(M))
        if vals.size == 0:
            return vals, 0.0
        a = np.abs(vals)
        return vals, float(a.max()) if not np.isnan(a).any() else float("nan")

    def batch(self, Iset, Jset, M):
        M = int(M)
        if len(Iset) * len(Jset) == 0:
            return np.zeros((0,) * (M + 2))
        nl = len(Iset[0])
        nr = len(Jset[0])
        if nl + M + nr != self.L:
            raise ValueError("Invalid number of central indices")
        if M > 1:
            raise NotImplementedError("batch evaluation supports M = 0 or 1 centre legs")
        out, _ = self.pi(np.asarray(Iset, np.int32).reshape(len(Iset), nl),
                         np.asarray(Jset, np.int32).reshape(len(Jset), nr), M)
        return out.reshape((len(Iset),) + tuple(self.localdims[nl:nl + M]) + (len(Jset),), order="F")

