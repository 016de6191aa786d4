"""CachedFunction -- host mirror of src/cachedfunction.jl.

CachedFunction{ValueType}(f, localdims) (cachedfunction.jl:53-135) memoises f by an integer key
(key = sum((x .- 1) .* coeffs), coeffs = cumprod([1; localdims[1:end-1]]), :197-199). Python
integers are unbounded, so one key type serves every index space (the reference picks
UInt32 ... UInt256 by size, :121-135; `keytype` reports that choice).

Batch evaluation (:255-302) looks every point up and evaluates only the misses: through ONE
device batch call when f is a device evaluator (GPUBatchEvaluator / ComplexScaledEvaluator:
f.points), else by calling f point by point like the reference. As a TCI2 evaluator it supplies
Pi through pi(); the rrLU and factors then run on the device (tci_luci_h / tci_luci_c128_h).
"""
import math

import numpy as np


class CachedFunction:
    def __init__(self, f, localdims, valuetype=float):
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

    # -- reference API
    def key(self, x):
        """key(cf, indexset) (cachedfunction.jl:197-199); raises like the reference's bounds
        error for an index set of the wrong length."""
        x = [int(v) for v in x]
        if len(x) != self.L:
            raise ValueError(f"index set of length {len(x)} for a function of {self.L} legs")
        return sum((v - 1) * c for v, c in zip(x, self.coeffs))

    def haskey(self, x):
        return self.key(x) in self.cache

    def cacheddata(self):
        """cacheddata(cf) (:160-170): index set -> value."""
        out = {}
        for k, v in self.cache.items():
            x = []
            for d in self.localdims:
                x.append(k % d + 1)
                k //= d
            out[tuple(x)] = v
        return out

    def ncacheddata(self):
        return len(self.cache)

    def clearcache(self):
        """clearcache!(cf) (:305-308)."""
        self.cache.clear()

    def __call__(self, x, Jset=None, M=None):
        if Jset is not None:
            return self.batch(x, Jset, M)
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
