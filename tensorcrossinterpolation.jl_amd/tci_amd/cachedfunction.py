"""CachedFunction -- host mirror of src/cachedfunction.jl.

CachedFunction{ValueType}(f, localdims) (cachedfunction.jl:53-135) memoises f by an integer key
(key = sum((x .- 1) .* coeffs), coeffs = cumprod([1; localdims[1:end-1]]), :197-199). Python
integers are unbounded, so one key type serves every index space (the reference picks
UInt32 ... UInt256 by size, :121-135; `keytype` reports that choice).

Batch evaluation (:255-302) looks every point up and evaluates only the misses: through ONE
device batch call when f is a device evaluator (GPUBatchEvaluator / ComplexScaledEvaluator:
f.points), else by calling f point by point like the reference. As a TCI2 evaluator it supplies
Pi through pi(); the rrLU and factors then run on the device (tci_luci_h / tci_luci_c128_h).

Device memo: when f is a real device integrand (GPUBatchEvaluator) and the
keys fit 62 bits, the memo itself lives in HBM (tci_cache_*, tci_cache.hip): a Pi block is served
by one probe pass (hits straight into Pi), the batch's distinct misses evaluated in one batch
evaluation of f and inserted -- no host dictionary, no per-point traffic.
"""
import ctypes as C
import math

import numpy as np


class _DeviceMemo:
    """tci_cache over a context (owned by it: released before the context)."""

    def __init__(self, ctx, localdims):
        from . import _lib

        self.ctx, self._lib = ctx, _lib
        h = C.c_void_p()
        ld = np.ascontiguousarray(localdims, np.int32)
        ctx.check(ctx.lib.tci_cache_create(ctx.h, ld, len(ld), 4096, C.byref(h)))
        self.h = h
        ctx.own(self)

    def release(self):
        if getattr(self, "h", None) and self.ctx.alive:
            self.ctx.lib.tci_cache_destroy(self.h)
        self.h = None

    def size(self):
        n = C.c_int64()
        self.ctx.check(self.ctx.lib.tci_cache_size(self.h, C.byref(n)))
        return n.value

    def clear(self):
        self.ctx.check(self.ctx.lib.tci_cache_clear(self.h))

    def dump(self):
        n = C.c_int64()
        self.ctx.check(self.ctx.lib.tci_cache_dump_h(self.h, None, None, 0, C.byref(n)))
        keys = np.zeros(max(n.value, 1), np.int64)
        vals = np.zeros(max(n.value, 1))
        self.ctx.check(self.ctx.lib.tci_cache_dump_h(self.h, self._lib.ptr(keys), self._lib.ptr(vals), n.value,
                                                     C.byref(n)))
        return keys[: n.value], vals[: n.value]

    def lookup(self, X):
        """(found, values) of the points X (npts x L) -- one device probe, no table dump."""
        X = np.ascontiguousarray(X, np.int32)
        found = np.zeros(max(len(X), 1), np.int32)
        vals = np.zeros(max(len(X), 1))
        self.ctx.check(self.ctx.lib.tci_cache_lookup_h(self.h, self._lib.ptr(X), len(X), self._lib.ptr(found),
                                                       self._lib.ptr(vals)))
        return found[: len(X)].astype(bool), vals[: len(X)]

    def pi(self, f, I, J, M):
        """(Pi as a Fortran (|I| D) x |J| array, max|Pi|, number of misses evaluated)."""
        ctx, _lib = self.ctx, self._lib
        I = np.ascontiguousarray(I, np.int32)
        J = np.ascontiguousarray(J, np.int32)
        m, nl = I.shape
        n, nr = J.shape
        D = f.localdims[nl] if M == 1 else 1
        out = np.zeros((m * D, n), order="F")
        mx, nm = C.c_double(), C.c_int64()
        ctx.check(ctx.lib.tci_cache_batcheval_h(ctx.h, self.h, f.h, _lib.ptr(I), m, nl, _lib.ptr(J), n, nr, M,
                                                out.ctypes.data_as(C.c_void_p), max(m * D, 1), C.byref(mx),
                                                C.byref(nm)))
        return out, mx.value, nm.value


class CachedFunction:
    def __init__(self, f, localdims, valuetype=float, device_memo=None):
        """device_memo: None = on when f is a real device integrand and the keys fit 62 bits."""
        self.f = f
        self.localdims = [int(d) for d in localdims]
        self.L = len(self.localdims)
        self.valuetype = complex if valuetype in (complex, np.complex128) else float
        # not the fused complex device update (that is ComplexScaledEvaluator's): Pi comes from
        # pi() and is factorised by tci_luci_h / tci_luci_c128_h
        self.is_complex = False
        self.cache = {}
        self.coeffs = [1] * self.L
        for n in range(1, self.L):
            self.coeffs[n] = self.localdims[n - 1] * self.coeffs[n - 1]
        log2space = sum(math.log2(d) for d in self.localdims)
        self.keytype = ("UInt32" if log2space < 31 else "UInt64" if log2space < 63 else
                        "UInt128" if log2space < 127 else "UInt256+")
        self.ctx = getattr(f, "ctx", None)
        self.nmiss_last = 0
        capable = (hasattr(f, "h") and not getattr(f, "is_complex", False) and self.valuetype is float
                   and log2space < 62.5)
        if device_memo and not capable:
            raise ValueError("device_memo needs a real device integrand and keys below 2^62")
        self._memo = _DeviceMemo(f.ctx, self.localdims) if (capable and device_memo is not False) else None

    # -- reference API
    def key(self, x):
        """key(cf, indexset) (cachedfunction.jl:197-199); raises like the reference's bounds
        error for an index set of the wrong length."""
        x = [int(v) for v in x]
        if len(x) != self.L:
            raise ValueError(f"index set of length {len(x)} for a function of {self.L} legs")
        return sum((v - 1) * c for v, c in zip(x, self.coeffs))

    def haskey(self, x):
        if self._memo is not None:
            self.key(x)  # argument check
            return bool(self._memo.lookup(np.asarray([x], np.int32).reshape(1, self.L))[0][0])
        return self.key(x) in self.cache

    def cacheddata(self):
        """cacheddata(cf) (:160-170): index set -> value."""
        out = {}
        if self._memo is not None:
            keys, vals = self._memo.dump()
            items = zip((int(k) for k in keys), (float(v) for v in vals))
        else:
            items = self.cache.items()
        for k, v in items:
            x = []
            for d in self.localdims:
                x.append(k % d + 1)
                k //= d
            out[tuple(x)] = v
        return out

    def ncacheddata(self):
        return self._memo.size() if self._memo is not None else len(self.cache)

    def clearcache(self):
        """clearcache!(cf) (:305-308)."""
        if self._memo is not None:
            self._memo.clear()
        self.cache.clear()

    def __call__(self, x, Jset=None, M=None):
        if Jset is not None:
            return self.batch(x, Jset, M)
        if self._memo is not None:
            return float(self.points(np.asarray([x]))[0])
        k = self.key(x)
        if k not in self.cache:
            self.cache[k] = self._eval(np.asarray([x], np.int64))[0]
        return self.cache[k]

    # -- evaluation of misses
    def _eval(self, X):
        if hasattr(self.f, "points"):  # device evaluator: one batch call
            vals = np.asarray(self.f.points(np.asarray(X, np.int32)))
        else:
            vals = np.array([self.f([int(v) for v in x]) for x in X])
        return [self.valuetype(v) for v in vals]

    def points(self, X):
        X = np.asarray(X, np.int64).reshape(-1, self.L)
        if self._memo is not None:
            out, _, self.nmiss_last = self._memo.pi(self.f, np.zeros((1, 0), np.int32), X.astype(np.int32), 0)
            return out[0, :].copy()
        if self.keytype in ("UInt32", "UInt64"):
            keys = ((X - 1) * np.asarray(self.coeffs, np.int64)).sum(1)
        else:  # beyond int64: exact Python integers
            keys = (X - 1).astype(object) @ np.asarray(self.coeffs, dtype=object)
        keys = [int(k) for k in keys]
        miss = [i for i, k in enumerate(keys) if k not in self.cache]
        # first occurrence only (a point may repeat within one batch)
        seen, first = set(), []
        for i in miss:
            if keys[i] not in seen:
                seen.add(keys[i])
                first.append(i)
        if first:
            for i, v in zip(first, self._eval(X[first])):
                self.cache[keys[i]] = v
        dt = np.complex128 if self.valuetype is complex else np.float64
        return np.array([self.cache[k] for k in keys], dtype=dt)

    def pi(self, I, J, M=0):
        """(|I| * D) x |J| Fortran matrix of f over I x (centre) x J and max|.| (util.jl:34)."""
        I = np.asarray(I, np.int64)
        J = np.asarray(J, np.int64)
        m, nl = I.shape
        n, nr = J.shape
        D = self.localdims[nl] if M == 1 else 1
        if self._memo is not None and m * D * n > 0:
            out, mx, self.nmiss_last = self._memo.pi(self.f, I, J, M)
            return out, mx
        if m * D * n == 0:
            dt = np.complex128 if self.valuetype is complex else np.float64
            return np.zeros((m * D, n), dt), 0.0
        # element (i + m * c, j), i fastest (batcheval.jl:157-171)
        ii = np.tile(np.arange(m), D * n)
        cc = np.tile(np.repeat(np.arange(D), m), n)
        jj = np.repeat(np.arange(n), m * D)
        parts = [I[ii]]
        if M == 1:
            parts.append((cc + 1)[:, None])
        parts.append(J[jj])
        X = np.concatenate(parts, axis=1)
        vals = self.points(X)
        out = vals.reshape((m * D, n), order="F")
        return out, float(np.max(np.abs(out)))  # NaN propagates like Base.max

    def batch(self, Iset, Jset, M):
        """(cf)(leftindexset, rightindexset, Val(M)) (cachedfunction.jl:255-302)."""
        M = int(M)
        if len(Iset) * len(Jset) == 0:
            return np.zeros((0,) * (M + 2))
        nl = len(Iset[0])
        nr = len(Jset[0])
        if nl + M + nr != self.L:
            raise ValueError("Invalid number of central indices")
        if M > 1:
            raise NotImplementedError("batch evaluation supports M = 0 or 1 centre legs")
        out, _ = self.pi(np.asarray(Iset, np.int64).reshape(len(Iset), nl),
                         np.asarray(Jset, np.int64).reshape(len(Jset), nr), M)
        return out.reshape((len(Iset),) + tuple(self.localdims[nl:nl + M]) + (len(Jset),), order="F")
