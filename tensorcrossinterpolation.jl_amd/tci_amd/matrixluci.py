"""MatrixLUCI on the GPU -- host-side mirror of src/matrixluci.jl.

MatrixLUCI(A; maxrank, reltol, abstol, leftorthogonal) (matrixluci.jl:55-57) factorises A with the
device rrLU and computes left/right factors (matrixluci.jl:256-283) with device TRSM/GEMM
kernels; rowindices/colindices are 1-based like the reference.
"""
import ctypes as C

import numpy as np

from . import _lib
from .matrixlu import INT64_MAX


class MatrixLUCI:
    """mutable struct MatrixLUCI{T} (matrixluci.jl:32-34), factors materialised on construction."""

    def __init__(self, A, maxrank=INT64_MAX, reltol=1e-14, abstol=0.0, leftorthogonal=True, ctx=None):
        ctx = ctx or _lib.context()
        cplx = np.iscomplexobj(A)  # MatrixLUCI{ComplexF64}: tci_luci_c128_h
        dt = np.complex128 if cplx else np.float64
        A = np.asfortranarray(np.asarray(A, dtype=dt))
        m, n = A.shape
        mr = int(max(min(int(maxrank), m, n), 0))
        rowidx = np.zeros(max(mr, 1), np.int64)
        colidx = np.zeros(max(mr, 1), np.int64)
        pe = np.zeros(mr + 1)
        lf = np.zeros(max(m * mr, 1), dt)
        rf = np.zeros(max(mr * n, 1), dt)
        npv = C.c_int64()
        entry = ctx.lib.tci_luci_c128_h if cplx else ctx.lib.tci_luci_h
        ctx.check(entry(ctx.h, _lib.ptr(A), m, n, max(m, 1), int(min(maxrank, INT64_MAX)),
                                     float(reltol), float(abstol), int(bool(leftorthogonal)),
                                     _lib.ptr(rowidx), _lib.ptr(colidx), _lib.ptr(pe), _lib.ptr(lf),
                                     _lib.ptr(rf), C.byref(npv)))
        k = npv.value
        self.shape = (m, n)
        self.leftorthogonal = bool(leftorthogonal)
        self.npivot = k
        self._rowindices = rowidx[:k].copy()
        self._colindices = colidx[:k].copy()
        self._pivoterrors = pe[: k + 1].copy()
        self._left = lf[: m * k].reshape((m, k), order="F").copy()
        self._right = rf[: k * n].reshape((k, n), order="F").copy()

    def size(self, dim=None):
        if dim is None:
            return self.shape
        return self.shape[dim - 1] if dim in (1, 2) else 1

    def npivots(self):
        return self.npivot

    def rowindices(self):
        return self._rowindices

    def colindices(self):
        return self._colindices

    def left(self):
        """left(luci) (matrixluci.jl:256-262)."""
        return self._left

    def right(self):
        """right(luci) (matrixluci.jl:277-283)."""
        return self._right

    def pivoterrors(self):
        return self._pivoterrors

    def lastpivoterror(self):
        return float(self._pivoterrors[-1])
