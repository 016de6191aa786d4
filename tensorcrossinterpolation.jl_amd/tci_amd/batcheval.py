"""Batch evaluation on the GPU -- host-side mirror of src/batcheval.jl and the BatchEvaluator
plugin type (cachedtensortrain.jl:31).

The reference's `f` is arbitrary Julia; a device kernel needs it as data, so integrands come from
a catalog (DESIGN.md "Integrand catalog"). `GPUBatchEvaluator` is the drop-in for a
`BatchEvaluator{Float64}`: it is callable on one MultiIndex (f(x)) and on
(Iset, Jset, M) like `(f)(Iset, Jset, Val(M))` (docs/src/index.md:174-243), returning arrays of
shape (|Iset|, d_{nl+1..nl+M}..., |Jset|) in column-major (Fortran) order.
"""
import ctypes as C
import math

import numpy as np

from . import _lib

F_SUM, F_LORENTZ, F_TABLE, F_GAUSS, F_GAUSSMIX, F_QOSC, F_QEXP, F_TT, F_CP, F_MPO = range(10)


def _as_index_table(sets, width):
    """Vector{MultiIndex} -> (count, width) int32 C-contiguous table (1-based values)."""
    a = np.asarray(sets, dtype=np.int32)
    if a.size == 0:
        return np.zeros((len(sets) if hasattr(sets, "__len__") else 0, width), np.int32)
    return np.ascontiguousarray(a.reshape(-1, width))


class GPUBatchEvaluator:
    """A BatchEvaluator{Float64} whose batch method runs on the GPU."""

    def __init__(self, kind, params, localdims, ctx=None, name=None):
        self.ctx = ctx or _lib.context()
        self.kind = int(kind)
        self.params = np.ascontiguousarray(np.asarray(params if params is not None else [], np.float64))
        self.localdims = [int(d) for d in localdims]
        self.L = len(self.localdims)
        self.name = name or f"kind{kind}"
        h = C.c_void_p()
        p = self.params if self.params.size else np.zeros(1)
        self.ctx.check(self.ctx.lib.tci_func_create(self.ctx.h, self.kind, _lib.ptr(p), int(self.params.size),
                                                    np.ascontiguousarray(self.localdims, np.int32), self.L,
                                                    C.byref(h)))
        self.h = h
        self.ctx.own(self)

    def release(self):
        if getattr(self, "h", None) and self.ctx.alive:
            self.ctx.lib.tci_func_destroy(self.h)
        self.h = None

    def __del__(self):
        try:
            self.release()
        except Exception:
            pass

    # -- single point, (bf::BatchEvaluatorAdapter)(indexset) (batcheval.jl:67-69)
    def __call__(self, x, Jset=None, M=None):
        if Jset is not None:
            return self.batch(x, Jset, M)
        x = np.asarray(x, np.int32).reshape(1, self.L)
        out, _ = self.pi(x, np.zeros((1, 0), np.int32))
        return float(out[0, 0])

    def points(self, X):
        """f at each row of X (count x L) -> vector (one device call)."""
        X = np.ascontiguousarray(np.asarray(X, np.int32).reshape(-1, self.L))
        out, _ = self.pi(X, np.zeros((1, 0), np.int32))
        return out[:, 0].copy()

    def pi(self, I, J, M=0):
        """Raw batch evaluation: (|I| * D) x |J| Fortran matrix and max|.| (util.jl:34)."""
        I = np.ascontiguousarray(np.asarray(I, np.int32))
        J = np.ascontiguousarray(np.asarray(J, np.int32))
        m, nl = I.shape
        n, nr = J.shape
        D = self.localdims[nl] if M == 1 else 1
        out = np.zeros(max(m * D * n, 1))
        mx = C.c_double()
        self.ctx.check(self.ctx.lib.tci_batcheval_h(self.ctx.h, self.h, _lib.ptr(I), m, nl, _lib.ptr(J), n, nr,
                                                    int(M), _lib.ptr(out), max(m * D, 1), C.byref(mx)))
        return out[: m * D * n].reshape((m * D, n), order="F"), mx.value

    def batch(self, Iset, Jset, M):
        """(f)(Iset, Jset, Val(M)) -> Array{Float64, M+2} (docs/src/index.md:174-243)."""
        M = int(M)
        if len(Iset) * len(Jset) == 0:
            return np.zeros((0,) * (M + 2))
        nl = len(Iset[0])
        nr = len(Jset[0])
        if nl + M + nr != self.L:
            raise ValueError("Invalid number of central indices")
        if M > 1:
            raise NotImplementedError("GPU batch evaluation supports M = 0 or 1 centre legs")
        I = _as_index_table(Iset, nl)
        J = _as_index_table(Jset, nr)
        out, _ = self.pi(I, J, M)
        shape = (len(Iset),) + tuple(self.localdims[nl:nl + M]) + (len(Jset),)
        return out.reshape(shape, order="F")


class ComplexScaledEvaluator:
    """A BatchEvaluator{ComplexF64}: coeff * f(x) over a real device integrand f, evaluated on the
    GPU (tci_batcheval_c128_h / tci_update_pivots_c128_h). The complex Lorentzian of
    test_tensorci2.jl:246-249, coeff ./ (sum(v.^2) + 1), is ComplexScaledEvaluator(coeff,
    lorentz(localdims)) (values agree with Julia's coeff / x to the last ulp of the product
    coeff * (1 / x))."""

    is_complex = True

    def __init__(self, coeff, f):
        self.coeff = complex(coeff)
        self.f = f
        self.localdims = list(f.localdims)
        self.L = f.L
        self.ctx = f.ctx

    def __call__(self, x, Jset=None, M=None):
        if Jset is not None:
            return self.batch(x, Jset, M)
        return complex(self.points(np.asarray(x, np.int32).reshape(1, self.L))[0])

    def points(self, X):
        X = np.ascontiguousarray(np.asarray(X, np.int32).reshape(-1, self.L))
        out, _ = self.pi(X, np.zeros((1, 0), np.int32))
        return out[:, 0].copy()

    def pi(self, I, J, M=0, want_values=True):
        """(|I| * D) x |J| complex Fortran matrix (None unless want_values) and max|.|."""
        I = np.ascontiguousarray(np.asarray(I, np.int32))
        J = np.ascontiguousarray(np.asarray(J, np.int32))
        m, nl = I.shape
        n, nr = J.shape
        D = self.localdims[nl] if M == 1 else 1
        out = np.zeros(max(m * D * n, 1), np.complex128) if want_values else None
        mx = C.c_double()
        self.ctx.check(self.ctx.lib.tci_batcheval_c128_h(
            self.ctx.h, self.f.h, self.coeff.real, self.coeff.imag, _lib.ptr(I), m, nl, _lib.ptr(J), n, nr,
            int(M), _lib.ptr(out), C.byref(mx)))
        if out is None:
            return None, mx.value
        return out[: m * D * n].reshape((m * D, n), order="F"), mx.value

    def batch(self, Iset, Jset, M):
        M = int(M)
        if len(Iset) * len(Jset) == 0:
            return np.zeros((0,) * (M + 2), np.complex128)
        nl = len(Iset[0])
        nr = len(Jset[0])
        if nl + M + nr != self.L:
            raise ValueError("Invalid number of central indices")
        if M > 1:
            raise NotImplementedError("GPU batch evaluation supports M = 0 or 1 centre legs")
        out, _ = self.pi(_as_index_table(Iset, nl), _as_index_table(Jset, nr), M)
        shape = (len(Iset),) + tuple(self.localdims[nl:nl + M]) + (len(Jset),)
        return out.reshape(shape, order="F")


# ------------------------------------------------------------------ catalog
def lorentz(localdims, coeff=1.0, **kw):
    """f(v) = coeff / (sum(v.^2) + 1): README.md:21-29, test_tensorci2.jl:247-250."""
    return GPUBatchEvaluator(F_LORENTZ, [coeff], localdims, name="lorentz", **kw)


def sum_(localdims, **kw):
    """f(x) = sum(x) (test_batcheval.jl:19)."""
    return GPUBatchEvaluator(F_SUM, [], localdims, name="sum", **kw)


def table(T, **kw):
    """f(x) = T[x...] for a dense column-major tensor T."""
    T = np.asarray(T, np.float64)
    return GPUBatchEvaluator(F_TABLE, T.ravel(order="F"), list(T.shape), name="table", **kw)


def gauss(localdims, a, c, **kw):
    """f(x) = exp(-(a * sum((x .- c).^2))): the separable Gaussian of BASELINE config 3."""
    return GPUBatchEvaluator(F_GAUSS, [a, c], localdims, name="gauss", **kw)


def gaussmix(localdims, a, centres, weights, **kw):
    """f(x) = sum_k w_k exp(-(a * sum((x .- c_k).^2))): a non-separable load for config 3."""
    centres = np.asarray(centres, np.float64)
    K = centres.shape[0]
    p = np.concatenate([[K, a], centres.ravel(), np.asarray(weights, np.float64)])
    return GPUBatchEvaluator(F_GAUSSMIX, p, localdims, name="gaussmix", **kw)


QOSC_PARAMS = [10.0, 2 * math.pi * 100, 1.1]  # exp(-10x) sin(2 pi 100 x^1.1), test_tensorci2.jl:437


def quantics_osc(R, params=None, **kw):
    """Quantics grid x = (i-1)/2^R on [0,1) (QuanticsGrids.DiscretizedGrid{1}(R, 0, 1)),
    f = exp(-p0 x) sin(p1 x^p2): the reference's "nasty function" (test_tensorci2.jl:437)."""
    return GPUBatchEvaluator(F_QOSC, params or QOSC_PARAMS, [2] * R, name="quantics_osc", **kw)


def quantics_exp(R, a=1.0, b=1.0, c=0.0, d=0.0, **kw):
    """f = a exp(-b x) + c exp(-d x) on the quantics grid (test_tensorci2.jl:65, :157)."""
    return GPUBatchEvaluator(F_QEXP, [a, b, c, d], [2] * R, name="quantics_exp", **kw)


def tensortrain_function(cores, **kw):
    """f(x) = T1[:, x1, :] ... TL[:, xL, :] (a TensorTrain/TTCache used as f, test_tensorci2.jl:477)."""
    bd = [cores[0].shape[0]] + [c.shape[2] for c in cores]
    p = np.concatenate([np.asarray(bd, np.float64)] + [np.asarray(c, np.float64).ravel(order="F") for c in cores])
    return GPUBatchEvaluator(F_TT, p, [c.shape[1] for c in cores], name="tt", **kw)


def cp_function(g, **kw):
    """f(x) = sum_k prod_t g[k][t][x_t - 1]: the CP-rank-K synthetic of BASELINE config 5
    (SURVEY.md 8(d)). g: array (K, L, dmax); leg t uses g[:, t, :localdims[t]]."""
    g = np.asarray(g, np.float64)
    K, L, dmax = g.shape
    localdims = kw.pop("localdims", [dmax] * L)
    p = np.concatenate([[K, dmax], g.ravel(order="C")])
    return GPUBatchEvaluator(F_CP, p, localdims, name="cp", **kw)


def quantics_bits(x, R):
    """QuanticsGrids origcoord_to_quantics for DiscretizedGrid{1}(R, 0, 1) (1-based bits)."""
    i = int(np.floor(x * 2 ** R))
    return [((i >> (R - 1 - t)) & 1) + 1 for t in range(R)]
