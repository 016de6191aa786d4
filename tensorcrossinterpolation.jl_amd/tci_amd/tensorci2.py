"""TCI2 driver -- host-side mirror of src/tensorci2.jl (plus the helpers it calls from
globalsearch.jl, util.jl and sweepstrategies.jl), with the hot path on the GPU.

This is what the Julia shim of INTEGRATION.md does inside Julia: the driver logic stays the
reference's, and every Pi assembly + rrLU + MatrixLUCI of `updatepivots!` / `sweep1site!`, every
`setsitetensor!` solve, runs in libtci_hip.so with Pi resident in HBM (tci_update_pivots_h,
tci_sitetensor_h). Only index sets, pivot errors and site tensors cross PCIe.

Conventions: sites/bonds are 1-based in this API like the reference (b in 1..L-1); index sets
are (count, width) int32 arrays of 1-based local indices.
"""
import contextlib
import ctypes as C
import os

import numpy as np

from . import _lib
from .batcheval import GPUBatchEvaluator

INT64_MAX = np.iinfo(np.int64).max


# ------------------------------------------------------------------ helpers
_BIG_FREE = 16 << 20  # site tensors at least this large are recycled


class _BufferPool:
    """Flat float64 buffers of large device -> host site tensors, recycled. Config 5 replaces 12
    tensors of up to 268 MB every iteration: freeing them (munmap) and faulting fresh pages in for
    the next ones cost ~0.3 s of its 21 s. A replaced tensor's buffer is taken back only when
    nothing else can see it -- the buffer came from this pool, the replaced array is a view whose
    only owner was the TensorCI2, and no other view of the buffer is alive -- so recycling is never
    observable. Bounded (_CAP bytes); anything else is simply dropped."""
    _CAP = 16 << 30

    def __init__(self):
        self.free = {}  # size -> [buffers]
        self.bytes = 0
        self.ids = set()  # ids of live buffers handed out by take()

    def take(self, n):
        lst = self.free.get(n)
        if lst:
            buf = lst.pop()
            self.bytes -= buf.nbytes
        else:
            buf = np.empty(max(n, 1))
        if buf.nbytes >= _BIG_FREE:
            self.ids.add(id(buf))
        return buf

    def give_back(self, arrays):
        import sys
        for i in range(len(arrays)):
            a = arrays[i]
            arrays[i] = None
            if not isinstance(a, np.ndarray) or a.nbytes < _BIG_FREE:
                continue
            root = a.base
            # the array (this local, getrefcount's argument) and its buffer (the array's .base, this
            # local, getrefcount's argument): any further reference means someone else holds it
            if (not isinstance(root, np.ndarray) or root.base is not None or id(root) not in self.ids
                    or sys.getrefcount(a) > 2 or sys.getrefcount(root) > 3):
                continue
            del a
            if self.bytes + root.nbytes > self._CAP:
                self.ids.discard(id(root))
                continue
            self.free.setdefault(root.size, []).append(root)
            self.bytes += root.nbytes


_POOL = _BufferPool()


def jl_max(x, y):
    """Base.max for Float64 (NaN-propagating, max(-0.0, 0.0) == 0.0)."""
    if (y > x) or (np.signbit(y) < np.signbit(x)):
        return x if np.isnan(x) else y
    return y if np.isnan(y) else x


def maxabs(maxval, value):
    """maxabs(maxval, updates) (util.jl:34-43) given max|updates| computed on the device."""
    return jl_max(abs(maxval), abs(value))


def kronecker_right(Iset, localdim):
    """kronecker(Iset, localdim) (tensorci2.jl:512-517): [is..., j], Iset fastest."""
    n, w = Iset.shape
    left = np.tile(Iset, (localdim, 1))
    loc = np.repeat(np.arange(1, localdim + 1, dtype=np.int32), n)[:, None]
    return np.ascontiguousarray(np.concatenate([left, loc], axis=1), dtype=np.int32)


def kronecker_left(localdim, Jset):
    """kronecker(localdim, Jset) (tensorci2.jl:524-529): [i, js...], i fastest."""
    n, w = Jset.shape
    loc = np.tile(np.arange(1, localdim + 1, dtype=np.int32), n)[:, None]
    right = np.repeat(Jset, localdim, axis=0)
    return np.ascontiguousarray(np.concatenate([loc, right], axis=1), dtype=np.int32)


def union_sets(a, b):
    """Julia union(a, b) on Vector{MultiIndex}: first-seen order, deduplicated."""
    if b is None or len(b) == 0:
        cat = a
    else:
        cat = np.concatenate([a, b], axis=0)
    if len(cat) == 0:
        return np.ascontiguousarray(cat, np.int32)
    if cat.shape[1] == 0:
        return np.zeros((1, 0), np.int32)
    cat = np.ascontiguousarray(cat, np.int32)
    keys = cat.view(np.dtype((np.void, 4 * cat.shape[1]))).ravel()
    if len(keys) <= 4096:  # small sets (every TCI2 bond at low rank): one dict pass
        seen = {}
        for i, k in enumerate(keys.tolist()):
            seen.setdefault(k, i)
        if len(seen) == len(keys):
            return cat
        return cat[np.fromiter(seen.values(), np.int64, len(seen))]
    _, first = np.unique(keys, return_index=True)
    return cat[np.sort(first)]


def pushunique(s, e):
    """pushunique! (util.jl:94-98) for one MultiIndex."""
    e = np.asarray(e, np.int32).reshape(1, -1)
    if len(s) and (s.shape[1] == 0 or np.any(np.all(s == e, axis=1))):
        return s
    return np.concatenate([s, e], axis=0)


def forwardsweep(sweepstrategy, iteration):
    """forwardsweep (sweepstrategies.jl:41-50)."""
    return sweepstrategy == "forward" or (sweepstrategy == "backandforth" and iteration % 2 == 1)


def convergencecriterion(ranks, errors, nglobalpivots, tolerance, maxbonddim, ncheckhistory,
                         checkconvglobalpivot=True):
    """convergencecriterion (tensorci2.jl:947-966)."""
    if len(errors) < ncheckhistory:
        return False
    lastranks = list(ranks[len(ranks) - ncheckhistory:])
    lastngp = list(nglobalpivots[len(nglobalpivots) - ncheckhistory:])
    lasterr = list(errors[len(errors) - ncheckhistory:])
    return (all(e < tolerance for e in lasterr)
            and (all(g == 0 for g in lastngp) if checkconvglobalpivot else True)
            and min(lastranks) == lastranks[-1]) or all(r >= maxbonddim for r in lastranks)


# ---------------------------------------------------------------- TensorCI2
class TensorCI2:
    """mutable struct TensorCI2{ValueType} (tensorci2.jl:50-93) for ValueType = Float64."""

    def __init__(self, localdims):
        localdims = [int(d) for d in localdims]
        if len(localdims) <= 1:
            raise ValueError("localdims should have at least 2 elements!")
        n = len(localdims)
        self.localdims = localdims
        # the index sets may live in the native object between native sweeps (_native_* below):
        # _py_stale = the native copy is newer (pulled on first access), _native_dirty = the Python
        # copy may have changed since the last push
        self._py_stale = False
        self._native_dirty = True
        self.Iset = [np.zeros((0, b), np.int32) for b in range(n)]
        self.Jset = [np.zeros((0, n - 1 - b), np.int32) for b in range(n)]
        self.sitetensors = [np.zeros((0, d, 0)) for d in localdims]
        self.pivoterrors = np.zeros(0)
        self.bonderrors = np.zeros(n - 1)
        self.maxsamplevalue = 0.0
        self.Iset_history = []  # only the last entry is ever read (tensorci2.jl:1214-1216)
        self.Jset_history = []

    @classmethod
    def from_function(cls, f, localdims, initialpivots=None):
        """TensorCI2{V}(func, localdims, initialpivots) (tensorci2.jl:105-116)."""
        tci = cls(localdims)
        L = len(tci.localdims)
        if initialpivots is None:
            initialpivots = [[1] * L]
        piv = np.asarray(initialpivots, np.int32).reshape(-1, L)
        tci.addglobalpivots(piv)
        vals = f.points(piv)
        mx = None
        for v in np.abs(vals):
            mx = v if mx is None else jl_max(mx, v)
        tci.maxsamplevalue = float(mx)
        if not abs(tci.maxsamplevalue) > 0.0:
            raise RuntimeError("maxsamplevalue is zero!")
        tci.invalidatesitetensors()
        return tci

    @classmethod
    def from_sets(cls, f, localdims, Iset, Jset):
        """TensorCI2{V}(func, localdims, Iset, Jset) (tensorci2.jl:123-137)."""
        tci = cls(localdims)
        tci.Iset = [np.ascontiguousarray(np.asarray(s, np.int32).reshape(len(s), b)) for b, s in enumerate(Iset)]
        n = len(tci.localdims)
        tci.Jset = [np.ascontiguousarray(np.asarray(s, np.int32).reshape(len(s), n - 1 - b)) for b, s in enumerate(Jset)]
        pivots = reconstractglobalpivotsfromijset(tci.localdims, tci.Iset, tci.Jset)
        vals = f.points(pivots)
        mx = None
        for v in np.abs(vals):
            mx = v if mx is None else jl_max(mx, v)
        tci.maxsamplevalue = float(mx)
        if not abs(tci.maxsamplevalue) > 0.0:
            raise RuntimeError("maxsamplevalue is zero!")
        tci.invalidatesitetensors()
        return tci

    # -- index sets (lazily synchronised with the native object)
    def _sets_get(name):
        def get(self):
            if self._py_stale:
                self._native_pull_sets()
            self._native_dirty = True  # the caller may modify what it gets
            return self.__dict__[name]

        def put(self, v):
            if self._py_stale:
                self._native_pull_sets()
            self.__dict__[name] = v
            self._native_dirty = True
        return property(get, put)

    Iset = _sets_get("_Iset")
    Jset = _sets_get("_Jset")
    Iset_history = _sets_get("_Iset_history")
    Jset_history = _sets_get("_Jset_history")
    del _sets_get

    # -- basic accessors (tensorci2.jl:189-289)
    def __len__(self):
        return len(self.localdims)

    def linkdims(self):
        if self._py_stale:  # the native object's counts: no pull of the sets themselves
            return [int(c) for c in self._native_counts(0)[1:]]
        return [len(self.Iset[b + 1]) for b in range(len(self) - 1)]

    def rank(self):
        return max(self.linkdims()) if len(self) > 1 else 0

    def invalidatesitetensors(self):
        old = list(self.sitetensors)
        for b in range(len(self)):
            self.sitetensors[b] = np.zeros((0, 0, 0))
        _POOL.give_back(old)

    def issitetensorsavailable(self):
        return all(t.size != 0 for t in self.sitetensors)

    def maxbonderror(self):
        m = self.bonderrors[0]
        for e in self.bonderrors[1:]:
            m = jl_max(m, e)
        return float(m)

    def pivoterror(self):
        return self.maxbonderror()

    def updatepivoterror(self, errors):
        """updatepivoterror! (tensorci2.jl:252-260): elementwise max over zero-padded vectors."""
        a, b = self.pivoterrors, np.asarray(errors, float)
        n = max(len(a), len(b))
        out = np.zeros(n)
        for i in range(n):
            out[i] = jl_max(a[i] if i < len(a) else 0.0, b[i] if i < len(b) else 0.0)
        self.pivoterrors = out

    def flushpivoterror(self):
        self.pivoterrors = np.zeros(0)

    def updateerrors(self, b, errors):
        """updateerrors! (tensorci2.jl:281-289); b is 1-based."""
        self.bonderrors[b - 1] = errors[-1]
        self.updatepivoterror(errors)

    def updatemaxsample(self, value):
        self.maxsamplevalue = maxabs(self.maxsamplevalue, value)

    def addglobalpivots(self, pivots):
        """addglobalpivots! (tensorci2.jl:335-357)."""
        L = len(self)
        piv = np.asarray(pivots, np.int32).reshape(-1, L) if len(pivots) else np.zeros((0, L), np.int32)
        for p in piv:
            for b in range(L):
                self.Iset[b] = pushunique(self.Iset[b], p[:b])
                self.Jset[b] = pushunique(self.Jset[b], p[b + 1:])
        if len(piv) > 0:
            self.invalidatesitetensors()

    def setsitetensor_(self, b, T):
        """setsitetensor!(tci, b, T) (tensorci2.jl:536-545); b is 1-based."""
        old = [self.sitetensors[b - 1]]
        self.sitetensors[b - 1] = np.asarray(T).reshape(
            (len(self.Iset[b - 1]), self.localdims[b - 1], len(self.Jset[b - 1])), order="F")
        _POOL.give_back(old)

    # -- hot path
    def updatepivots(self, b, f, leftorthogonal, reltol=1e-14, abstol=0.0, maxbonddim=INT64_MAX,
                     extraIset=None, extraJset=None, compute_factors=True):
        """updatepivots! (tensorci2.jl:825-930), :full pivot search; b is 1-based.

        Pi assembly, maxabs, rrLU and the MatrixLUCI factors run in one device call. When no
        caller can observe the site tensors this sets (sweep2site! with fillsitetensors=true
        overwrites them all), compute_factors=False skips the factor kernels; indices and errors
        are identical either way."""
        self.invalidatesitetensors()
        Icomb = union_sets(kronecker_right(self.Iset[b - 1], self.localdims[b - 1]), extraIset)
        Jcomb = union_sets(kronecker_left(self.localdims[b], self.Jset[b]), extraJset)
        noextra = (extraIset is None or len(extraIset) == 0) and (extraJset is None or len(extraJset) == 0)
        want = bool(compute_factors and noextra)
        res = update_pivots_device(f, Icomb, Jcomb, maxbonddim, reltol, abstol, leftorthogonal, want)
        self.updatemaxsample(res["maxabs"])
        self.Iset[b] = Icomb[res["rowidx"] - 1]
        self.Jset[b - 1] = Jcomb[res["colidx"] - 1]
        if want:
            self.setsitetensor_(b, res["left"])
            self.setsitetensor_(b + 1, res["right"])
        self.updateerrors(b, res["pivoterrors"])

    def setsitetensor(self, f, b, leftorthogonal=True, solve=True):
        """setsitetensor!(tci, f, b) (tensorci2.jl:599-629) on the device; b is 1-based.
        solve=False only updates maxsamplevalue from Pi1 (used when the solved tensor is
        unobservable because a later sweep overwrites it)."""
        if not leftorthogonal:
            raise ValueError("leftorthogonal==false is not supported!")
        p = b - 1
        Ib, Jb = self.Iset[p], self.Jset[p]
        last = b == len(self)
        Inext = None if last else self.Iset[p + 1]
        if not last and len(Inext) != len(Jb):
            raise RuntimeError(f"Pivot matrix at bond {b} is not square!")
        T, mx = sitetensor_device(f, Ib, Jb, Inext, solve)
        self.updatemaxsample(mx)
        if solve:
            self.setsitetensor_(b, T)
            return self.sitetensors[p]
        return None

    def fillsitetensors(self, f, solve=True):
        """fillsitetensors! (globalsearch.jl:202-208)."""
        for b in range(1, len(self) + 1):
            self.setsitetensor(f, b, solve=solve)

    def sweep1site(self, f, sweepdirection="forward", reltol=1e-14, abstol=0.0, maxbonddim=INT64_MAX,
                   updatetensors=True):
        """sweep1site! (tensorci2.jl:659-725)."""
        self.flushpivoterror()
        self.invalidatesitetensors()
        if sweepdirection not in ("forward", "backward"):
            raise ValueError(f"Unknown sweep direction {sweepdirection}: choose between :forward, :backward.")
        fwd = sweepdirection == "forward"
        L = len(self)
        if NATIVE_SWEEP and _native_ok(f) and self._sweep1site_native(f, fwd, reltol, abstol, maxbonddim,
                                                                        updatetensors):
            return
        bonds = range(1, L) if fwd else range(L, 1, -1)
        for b in bonds:
            p = b - 1
            if fwd:
                Is = kronecker_right(self.Iset[p], self.localdims[p])
                Js = self.Jset[p]
            else:
                Is = self.Iset[p]
                Js = kronecker_left(self.localdims[p], self.Jset[p])
            res = update_pivots_device(f, Is, Js, maxbonddim, reltol, abstol, fwd, updatetensors,
                                       want_left=fwd, want_right=not fwd)
            self.updatemaxsample(res["maxabs"])
            self.Iset[p + (1 if fwd else 0)] = Is[res["rowidx"] - 1]
            self.Jset[p - (0 if fwd else 1)] = Js[res["colidx"] - 1]
            if updatetensors:
                self.setsitetensor_(b, res["left"] if fwd else res["right"])
                if np.any(np.isnan(self.sitetensors[p])):
                    raise RuntimeError(f"Error: NaN in tensor T[{b}]")
            self.updateerrors(b - (0 if fwd else 1), res["pivoterrors"])
        if updatetensors:
            last = L if fwd else 1
            T, _ = sitetensor_device(f, self.Iset[last - 1], self.Jset[last - 1], None, True)
            self.setsitetensor_(last, T)

    def makecanonical(self, f, reltol=1e-14, abstol=0.0, maxbonddim=INT64_MAX):
        """makecanonical! (tensorci2.jl:738-749)."""
        self.sweep1site(f, "forward", reltol=0.0, abstol=0.0, maxbonddim=INT64_MAX, updatetensors=False)
        self.sweep1site(f, "backward", reltol=reltol, abstol=abstol, maxbonddim=maxbonddim, updatetensors=False)
        self.sweep1site(f, "forward", reltol=reltol, abstol=abstol, maxbonddim=maxbonddim, updatetensors=True)

    def addglobalpivots1sitesweep(self, f, pivots, reltol=1e-14, abstol=0.0, maxbonddim=INT64_MAX):
        """addglobalpivots1sitesweep! (tensorci2.jl:367-377)."""
        self.addglobalpivots(pivots)
        self.makecanonical(f, reltol=reltol, abstol=abstol, maxbonddim=maxbonddim)

    def sweep2site(self, f, niter, iter1=1, abstol=1e-8, maxbonddim=INT64_MAX, sweepstrategy="backandforth",
                   pivotsearch="full", verbosity=0, strictlynested=False, fillsitetensors=True,
                   lazy_sitetensors=False, native=None):
        """sweep2site! (tensorci2.jl:1195-1258). For a real device integrand the per-bond loop runs
        in C++ (tci_tci2_sweep2site, one ABI call per sweep; native=False forces this loop)."""
        if pivotsearch != "full":
            raise NotImplementedError("only pivotsearch=:full is implemented (the :rook search is random)")
        self.invalidatesitetensors()
        n = len(self)
        if native is not False and NATIVE_SWEEP and _native_ok(f) and fillsitetensors:
            # fillsitetensors! in the same device launch when it can: with the solves (the
            # reference's work, tci_tci2_sweep2site_fillsolve) or, lazy, only updatemaxsample! over
            # every site's Pi1 (tci_tci2_sweep2site_fill)
            done = self._sweep2site_native(f, niter, iter1, abstol, maxbonddim, sweepstrategy, strictlynested,
                                           fill="max" if lazy_sitetensors else "solve")
            if not done:
                self.fillsitetensors(f, solve=not lazy_sitetensors)
            return
        for it in range(iter1, iter1 + niter):
            extraI = [None] * n
            extraJ = [None] * n
            if not strictlynested and len(self.Iset_history) > 0:
                extraI = self.Iset_history[-1]
                extraJ = self.Jset_history[-1]
            self.Iset_history = [[s.copy() for s in self.Iset]]
            self.Jset_history = [[s.copy() for s in self.Jset]]
            self.flushpivoterror()
            # factors set here are always overwritten by fillsitetensors! below
            cf = not fillsitetensors
            if forwardsweep(sweepstrategy, it):
                for b in range(1, n):
                    self.updatepivots(b, f, True, abstol=abstol, maxbonddim=maxbonddim,
                                      extraIset=extraI[b], extraJset=extraJ[b - 1], compute_factors=cf)
            else:
                for b in range(n - 1, 0, -1):
                    self.updatepivots(b, f, False, abstol=abstol, maxbonddim=maxbonddim,
                                      extraIset=extraI[b], extraJset=extraJ[b - 1], compute_factors=cf)
        if fillsitetensors:
            self.fillsitetensors(f, solve=not lazy_sitetensors)

    def _native_handle(self, ctx):
        h = getattr(self, "_native_h", None)
        if h is None or getattr(self, "_native_ctx", None) is not ctx:
            if h is not None and self._py_stale:
                self._native_pull_sets()  # the newest sets live only in the old native object
                self._native_dirty = True  # ... so the new one must receive them
            h = C.c_void_p()
            ctx.check(ctx.lib.tci_tci2_create(ctx.h, len(self), np.ascontiguousarray(self.localdims, np.int32),
                                              C.byref(h)))
            self._native_h, self._native_ctx = h, ctx
            self._native_owner = ctx.own(_NativeTCI2(ctx, h))
        return h

    def _sweep1site_native(self, f, fwd, reltol, abstol, maxbonddim, updatetensors):
        """sweep1site! in one device launch (tci_tci2_sweep1site) when every bond fits the
        one-workgroup rrLU; False (state untouched) when the host loop has to run it."""
        ctx = f.ctx
        lib = ctx.lib
        n = len(self)
        h = self._native_handle(ctx)
        self._native_push(ctx, h)
        cap = n * 16384 if updatetensors else 0  # each site's tensor fits the small path's LDS
        tens = np.empty(max(cap, 1))
        offs = np.zeros(2 * n, np.int64)
        handled = C.c_int(0)
        with self._native_failure_sync(ctx, h):
            ctx.check(lib.tci_tci2_sweep1site(h, f.h, int(bool(fwd)), float(reltol), float(abstol),
                                              int(min(maxbonddim, INT64_MAX)), int(bool(updatetensors)),
                                              tens.ctypes.data_as(C.c_void_p), cap, offs.ctypes.data_as(C.c_void_p),
                                              C.byref(handled)))
        if not handled.value:
            return False
        self._native_pull(ctx, h)  # sweep1site! leaves the history alone (so does the kernel)
        if updatetensors:
            self._native_set_tensors(tens, offs)
        return True

    def _optimize_native(self, f, tol, maxbonddim, maxiter, ncheckhistory, normalizeerror, strictlynested, lazy):
        """optimize!'s loop and closing sweep1site! as one chain of device launches
        (tci_tci2_optimize_small). None when nothing ran on the device; else (iterations done, their
        errors, their ranks, loop ended, closing sweep done, the maxsample it normalised with)."""
        ctx = f.ctx
        lib = ctx.lib
        n = len(self)
        h = self._native_handle(ctx)
        self._native_push(ctx, h)
        cap = n * 16384
        tens = np.empty(cap)
        offs = np.zeros(2 * n, np.int64)
        errs = np.zeros(maxiter)
        rks = np.zeros(maxiter, np.int64)
        nd, ended, s1done = C.c_int32(), C.c_int32(), C.c_int32()
        errnorm, handled = C.c_double(), C.c_int(0)
        with self._native_failure_sync(ctx, h, hist=True):
            ctx.check(lib.tci_tci2_optimize_small(h, f.h, float(tol), int(min(maxbonddim, INT64_MAX)), int(maxiter),
                                                  int(ncheckhistory), int(bool(normalizeerror)),
                                                  int(bool(strictlynested)), int(not lazy),
                                                  tens.ctypes.data_as(C.c_void_p), cap,
                                                  offs.ctypes.data_as(C.c_void_p), errs.ctypes.data_as(C.c_void_p),
                                                  rks.ctypes.data_as(C.c_void_p), C.byref(nd), C.byref(ended),
                                                  C.byref(s1done), C.byref(errnorm), C.byref(handled)))
        if not handled.value:
            return None
        k = nd.value
        if k > 0:
            self._native_has_hist = True
        self._native_pull(ctx, h)
        self.invalidatesitetensors()
        if s1done.value:
            self._native_set_tensors(tens, offs)
        return (k, [float(x) for x in errs[:k]], [int(x) for x in rks[:k]], bool(ended.value), bool(s1done.value),
                float(errnorm.value))

    def _native_set_tensors(self, tens, offs):
        """setsitetensor! for every site from a native fill's packed output: the shapes from the
        native set counts, so the (still native-side) index sets are neither pulled nor marked as
        modified -- the next sweep does not have to push them back."""
        nI, nJ = self._native_counts(0), self._native_counts(1)
        for p in range(len(self)):
            o, c = int(offs[2 * p]), int(offs[2 * p + 1])
            shape = (int(nI[p]), int(self.localdims[p]), int(nJ[p]))
            if shape[0] * shape[1] * shape[2] != c:
                raise RuntimeError(f"native site tensor {p + 1}: {c} values for shape {shape}")
            self.sitetensors[p] = tens[o:o + c].reshape(shape, order="F")

    def _sweep2site_native(self, f, niter, iter1, abstol, maxbonddim, sweepstrategy, strictlynested,
                           fill=None):
        """The iterations in C++ / on the device (tci_tci2_sweep2site): the state goes in and comes
        back bank by bank (a few ABI calls, not one per set). fill: None, "max" (fillsitetensors!'s
        maxsample update only) or "solve" (fillsitetensors! with every site tensor solved, the
        reference's work). Returns whether that fill was done natively too."""
        ctx = f.ctx
        lib = ctx.lib
        h = self._native_handle(ctx)
        self._native_push(ctx, h)
        strat = {"backandforth": 0, "forward": 1, "backward": 2}[sweepstrategy]
        handled = C.c_int(0)
        mb = int(min(maxbonddim, INT64_MAX))
        n = len(self)
        if fill == "solve":
            cap = n * 16384  # each site's tensor fits the small path's LDS
            tens = np.empty(cap)
            offs = np.zeros(2 * n, np.int64)
            tp, op = tens.ctypes.data_as(C.c_void_p), offs.ctypes.data_as(C.c_void_p)
        with self._native_failure_sync(ctx, h, hist=niter > 0):
            if fill == "max" and niter > 0:
                ctx.check(lib.tci_tci2_sweep2site_fill(h, f.h, int(niter), int(iter1), float(abstol), mb, strat,
                                                       int(bool(strictlynested)), C.byref(handled)))
            elif fill == "solve" and niter > 0:
                ctx.check(lib.tci_tci2_sweep2site_fillsolve(h, f.h, int(niter), int(iter1), float(abstol), mb, strat,
                                                            int(bool(strictlynested)), tp, cap, op, C.byref(handled)))
            else:
                ctx.check(lib.tci_tci2_sweep2site(h, f.h, int(niter), int(iter1), float(abstol), mb, strat,
                                                  int(bool(strictlynested))))
                if fill == "max":
                    ctx.check(lib.tci_tci2_fill_maxsample(h, f.h, C.byref(handled)))
                elif fill == "solve":
                    ctx.check(lib.tci_tci2_fill_solve(h, f.h, tp, cap, op, C.byref(handled)))
        if niter > 0:
            self._native_has_hist = True  # every iteration starts a history
        self._native_pull(ctx, h)
        if fill == "solve" and handled.value:
            self._native_set_tensors(tens, offs)
        return bool(handled.value)

    @contextlib.contextmanager
    def _native_failure_sync(self, ctx, h, hist=False):
        """A native sweep that fails (a NaN, a host callback's error) has already updated the native
        sets in place, as the reference's sweep leaves the TensorCI2 half-updated when it throws: the
        Python mirror then follows the native state (pulled on first access) before re-raising, so
        the next push cannot resume from the stale Python copy."""
        try:
            yield
        except Exception:
            if hist:
                self._native_has_hist = True
            try:
                self._native_pull(ctx, h)
            except Exception:  # the original error is the one to report
                self._py_stale = True
                self._native_dirty = False
            raise

    def _native_counts(self, which):
        ctx = self._native_ctx
        counts = np.zeros(len(self), np.int64)
        ctx.check(ctx.lib.tci_tci2_get_sets(self._native_h, which, counts.ctypes.data_as(C.c_void_p), None, 0))
        return counts

    def _native_push(self, ctx, h):
        """The state into the native object, bank by bank (the sets only when the Python copy may
        have changed since the native object last had them)."""
        lib = ctx.lib
        if not self._native_dirty and getattr(self, "_native_synced_h", None) is h:
            self._native_push_errors(ctx, h)
            return

        def push(which, sets):
            counts = np.array([len(a) for a in sets], np.int64)
            parts = [np.ascontiguousarray(a, np.int32).ravel() for a in sets]
            packed = np.concatenate(parts) if parts else np.zeros(0, np.int32)
            packed = np.ascontiguousarray(packed, np.int32)
            ctx.check(lib.tci_tci2_set_sets(h, which, counts.ctypes.data_as(C.c_void_p),
                                            packed.ctypes.data_as(C.c_void_p)))

        push(0, self._Iset)
        push(1, self._Jset)
        if self._Iset_history:
            push(2, self._Iset_history[-1])
            push(3, self._Jset_history[-1])
        else:
            ctx.check(lib.tci_tci2_clear_history(h))
        self._native_has_hist = bool(self._Iset_history)
        self._native_dirty = False
        self._native_synced_h = h
        self._native_push_errors(ctx, h)

    def _native_push_errors(self, ctx, h):
        lib = ctx.lib
        pe = np.ascontiguousarray(self.pivoterrors, np.float64)
        ctx.check(lib.tci_tci2_set_errors(h, float(self.maxsamplevalue),
                                          np.ascontiguousarray(self.bonderrors, np.float64).ctypes.data_as(C.c_void_p),
                                          pe.ctypes.data_as(C.c_void_p), len(pe)))

    def _native_pull(self, ctx, h):
        """After a native sweep: errors and maxsamplevalue now; the sets when first read."""
        self._py_stale = True
        self._native_dirty = False
        self._native_pull_errors(ctx, h)

    def _native_pull_sets(self):
        ctx, h = self._native_ctx, self._native_h
        lib = ctx.lib
        n = len(self)
        widths = [list(range(n)), [n - 1 - p for p in range(n)]]

        def pull(which):
            counts = np.zeros(n, np.int64)
            ctx.check(lib.tci_tci2_get_sets(h, which, counts.ctypes.data_as(C.c_void_p), None, 0))
            w = widths[which % 2]
            tot = int(sum(int(c) * w[p] for p, c in enumerate(counts)))
            packed = np.zeros(max(tot, 1), np.int32)
            ctx.check(lib.tci_tci2_get_sets(h, which, counts.ctypes.data_as(C.c_void_p),
                                            packed.ctypes.data_as(C.c_void_p), len(packed)))
            out, o = [], 0
            for p, c in enumerate(counts):
                k = int(c) * w[p]
                out.append(packed[o:o + k].reshape(int(c), w[p]).copy())
                o += k
            return out

        d = self.__dict__
        d["_Iset"], d["_Jset"] = pull(0), pull(1)
        if self._native_has_hist:
            d["_Iset_history"], d["_Jset_history"] = [pull(2)], [pull(3)]
        else:
            d["_Iset_history"], d["_Jset_history"] = [], []
        self._py_stale = False

    def _native_pull_errors(self, ctx, h):
        lib = ctx.lib
        n = len(self)
        ms, npe = C.c_double(), C.c_int64()
        be = np.zeros(n - 1)
        pe = np.zeros(2048 + 1)
        ctx.check(lib.tci_tci2_errors(h, C.byref(ms), be.ctypes.data_as(C.c_void_p), pe.ctypes.data_as(C.c_void_p),
                                      len(pe), C.byref(npe)))
        if npe.value > len(pe):
            pe = np.zeros(npe.value)
            ctx.check(lib.tci_tci2_errors(h, C.byref(ms), be.ctypes.data_as(C.c_void_p),
                                          pe.ctypes.data_as(C.c_void_p), npe.value, C.byref(npe)))
        self.maxsamplevalue = ms.value
        self.bonderrors = be
        self.pivoterrors = pe[: npe.value].copy()

    def optimize(self, f, tolerance=None, pivottolerance=None, maxbonddim=INT64_MAX, maxiter=20,
                 sweepstrategy="backandforth", pivotsearch="full", verbosity=0, loginterval=10,
                 normalizeerror=True, ncheckhistory=3, globalpivotfinder=None, maxnglobalpivot=5,
                 nsearchglobalpivot=5, tolmarginglobalsearch=10.0, strictlynested=False,
                 checkbatchevaluatable=False, checkconvglobalpivot=True, rng=None, lazy_sitetensors=False):
        """optimize! (tensorci2.jl:1018-1172). Returns (ranks, errors ./ errornormalization).

        lazy_sitetensors (not a reference keyword; default False = the reference's work): with no
        global pivot search the site tensors that fillsitetensors! solves after every sweep2site!
        (tensorci2.jl:1254-1256, :599-629) are never read -- sweep1site! rebuilds all of them at the
        end -- so True skips their P evaluations and solves and keeps only updatemaxsample!. Ranks,
        errors, sets and the final tensors are identical; what differs is the work done and the
        number of f evaluations (visible to a counting or caching evaluator)."""
        errors, ranks, nglobalpivots = [], [], []
        # any BatchEvaluator is accepted (tensorci2.jl:1044): the device evaluators and every
        # HostFunctionEvaluator (pointwise, threaded or batch: it always exposes the batch interface)
        from .hostfunction import HostFunctionEvaluator
        if checkbatchevaluatable and not (isinstance(f, (GPUBatchEvaluator, HostFunctionEvaluator))
                                          or getattr(f, "is_batch", False)):
            raise RuntimeError("Function `f` is not batch evaluatable")
        if 0 < nsearchglobalpivot < maxnglobalpivot:
            raise RuntimeError("nsearchglobalpivot < maxnglobalpivot!")
        if pivottolerance is not None:
            if tolerance is not None and tolerance != pivottolerance:
                raise ValueError("Got different values for pivottolerance and tolerance in optimize!(TCI2). "
                                 "For TCI2, both of these options have the same meaning. Please assign only "
                                 "`tolerance`.")
            tol = pivottolerance
        elif tolerance is not None:
            tol = tolerance
        else:
            tol = 1e-8
        if maxbonddim >= INT64_MAX and tol <= 0:
            raise ValueError("Specify either tolerance > 0 or some maxbonddim; otherwise, the convergence "
                             "criterion is not reachable!")
        if globalpivotfinder is None:
            from .globalpivotfinder import DefaultGlobalPivotFinder
            finder = DefaultGlobalPivotFinder(nsearch=nsearchglobalpivot, maxnglobalpivot=maxnglobalpivot,
                                              tolmarginglobalsearch=tolmarginglobalsearch)
        else:
            finder = globalpivotfinder
        # The solved site tensors of fillsitetensors! are read only by a global pivot search;
        # with no search they are unobservable (sweep1site! below rebuilds all of them).
        searches = getattr(finder, "nsearch", 1) > 0
        lazy = bool(lazy_sitetensors) and not searches
        it0, loop_done = 1, False
        if (OPTIMIZE_CHAIN and NATIVE_SWEEP and _native_ok(f) and not searches and sweepstrategy == "backandforth"
                and pivotsearch == "full" and verbosity == 0 and 1 <= maxiter < 64 and ncheckhistory >= 1):
            # the whole loop (and sweep1site!) as one chain of device launches when every bond fits
            # the device-resident small sweep; the same iterations, tests and results as below
            r = self._optimize_native(f, tol, maxbonddim, maxiter, ncheckhistory, normalizeerror, strictlynested,
                                      lazy)
            if r is not None:
                nd, errs_d, rks_d, ended, s1done, errnorm = r
                errors.extend(errs_d)
                ranks.extend(rks_d)
                nglobalpivots.extend([0] * nd)
                if s1done:
                    self._sanitycheck()
                    en = errnorm if normalizeerror else 1.0
                    return ranks, [e / en for e in errors]
                it0, loop_done = nd + 1, ended
        for it in range(it0, maxiter + 1):
            if loop_done:
                break
            errornormalization = self.maxsamplevalue if normalizeerror else 1.0
            abstol = tol * errornormalization
            self.sweep2site(f, 2, iter1=1, abstol=abstol, maxbonddim=maxbonddim, pivotsearch=pivotsearch,
                            strictlynested=strictlynested, verbosity=verbosity, sweepstrategy=sweepstrategy,
                            fillsitetensors=True, lazy_sitetensors=lazy)
            errors.append(self.pivoterror())
            globalpivots = finder(self, f, abstol, verbosity=verbosity, rng=rng) if searches else []
            self.addglobalpivots(globalpivots)
            nglobalpivots.append(len(globalpivots))
            ranks.append(self.rank())
            if verbosity > 0 and it % loginterval == 0:
                print(f"iteration = {it}, rank = {ranks[-1]}, error= {errors[-1]}, "
                      f"maxsamplevalue= {self.maxsamplevalue}, nglobalpivot={len(globalpivots)}")
            if convergencecriterion(ranks, errors, nglobalpivots, abstol, maxbonddim, ncheckhistory,
                                    checkconvglobalpivot):
                break
        errornormalization = self.maxsamplevalue if normalizeerror else 1.0
        abstol = tol * errornormalization
        self.sweep1site(f, abstol=abstol, maxbonddim=maxbonddim)
        self._sanitycheck()
        return ranks, [e / errornormalization for e in errors]

    def _sanitycheck(self):
        """_sanitycheck (globalsearch.jl:226-233). (With the sets still native-side, their counts
        are read without pulling the sets.)"""
        if self._py_stale:
            nI, nJ = self._native_counts(0), self._native_counts(1)
            lens = [(int(nI[b]), int(nJ[b - 1])) for b in range(1, len(self))]
        else:
            lens = [(len(self.Iset[b]), len(self.Jset[b - 1])) for b in range(1, len(self))]
        for b, (i, j) in enumerate(lens, start=1):
            if i != j:
                raise RuntimeError(f"Pivot matrix at bond {b} is not square!")
        return True

    # -- tensor-train view (abstracttensortrain.jl:328-342, 428-441)
    def evaluate(self, idx):
        v = np.ones((1, 1))
        for p, i in enumerate(idx):
            v = v @ self.sitetensors[p][:, int(i) - 1, :]
        return complex(v[0, 0]) if np.iscomplexobj(v) else float(v[0, 0])

    def evaluate_many(self, X, ctx=None):
        """evaluate at every row of X in one device call (tci_tt_evaluate_h): the batched
        tensor-train evaluation of the global pivot search (globalpivotfinder.jl:236)."""
        X = np.ascontiguousarray(np.asarray(X, np.int32).reshape(-1, len(self)))
        if len(X) == 0:
            return np.zeros(0)
        ctx = ctx or _lib.context()
        dims = np.asarray(self.localdims, np.int32)
        bd = np.asarray([self.sitetensors[0].shape[0]] + [T.shape[2] for T in self.sitetensors], np.int32)
        if any(np.iscomplexobj(T) for T in self.sitetensors):  # TensorCI2{ComplexF64}
            cores = np.concatenate([np.asarray(T, np.complex128).ravel(order="F") for T in self.sitetensors])
            out = np.zeros(len(X), np.complex128)
            ctx.check(ctx.lib.tci_tt_evaluate_c128_h(ctx.h, len(self), _lib.ptr(dims), _lib.ptr(bd),
                                                     _lib.ptr(cores), cores.size, _lib.ptr(X), len(X),
                                                     _lib.ptr(out)))
            return out
        cores = np.concatenate([np.asarray(T, np.float64).ravel(order="F") for T in self.sitetensors])
        out = np.zeros(len(X))
        ctx.check(ctx.lib.tci_tt_evaluate_h(ctx.h, len(self), _lib.ptr(dims), _lib.ptr(bd), _lib.ptr(cores),
                                            cores.size, _lib.ptr(X), len(X), _lib.ptr(out)))
        return out

    def sum(self):
        v = np.ones((1, 1))
        for T in self.sitetensors:
            v = v @ T.sum(axis=1)
        return float(v[0, 0])


def reconstractglobalpivotsfromijset(localdims, Isets, Jsets):
    """reconstractglobalpivotsfromijset (tensorci2.jl:303-320)."""
    seen = set()
    out = []
    for i in range(len(Isets)):
        for I in Isets[i]:
            for J in Jsets[i]:
                for j in range(1, localdims[i] + 1):
                    e = tuple(int(x) for x in I) + (j,) + tuple(int(x) for x in J)
                    if e not in seen:
                        seen.add(e)
                        out.append(e)
    return np.asarray(out, np.int32)


# --------------------------------------------------------------- device calls
def _native_ok(f):
    """The native sweep driver takes a real device integrand (a GPUBatchEvaluator's tci_func)."""
    return (hasattr(f, "h") and getattr(f, "ctx", None) is not None and not getattr(f, "is_complex", False)
            and not getattr(f, "shard_rrlu", False)
            and type(f).__name__ in ("GPUBatchEvaluator", "HostFunctionEvaluator"))


class _NativeTCI2:
    """Owner of a tci_tci2 handle (released before its context)."""

    def __init__(self, ctx, h):
        self.ctx, self.h = ctx, h

    def release(self):
        if self.h and self.ctx.alive:
            self.ctx.lib.tci_tci2_destroy(self.h)  # host memory only: no HIP call
        self.h = None

    __del__ = release


# the native per-bond loop for device integrands (set False to run sweep2site's Python loop)
NATIVE_SWEEP = True
# optimize!'s whole loop as one chain of device launches where the small sweep takes every bond
# (set False, or TCI_OPT_CHAIN=0, for the per-iteration native calls)
OPTIMIZE_CHAIN = os.environ.get("TCI_OPT_CHAIN", "1") != "0"


def _ctx_of(f):
    ctx = getattr(f, "ctx", None) or getattr(getattr(f, "local", None), "ctx", None)
    return ctx or _lib.context()


def update_pivots_device(f, rows, cols, maxrank, reltol, abstol, leftorth, want_factors,
                         want_left=True, want_right=True):
    """One fused device call: Pi = f(rows x cols), maxabs, rrLU, pivots, MatrixLUCI factors.
    An evaluator that is not a GPUBatchEvaluator (e.g. a ShardedBatchEvaluator) supplies Pi
    through its pi() method; the factorisation then runs on this process's GPU."""
    if getattr(f, "is_complex", False):
        if getattr(f, "host_values", False):  # a complex batch computed on the host (pi())
            return _update_pivots_generic(f, rows, cols, maxrank, reltol, abstol, leftorth, want_factors,
                                          want_left, want_right)
        return _update_pivots_c128(f, rows, cols, maxrank, reltol, abstol, leftorth, want_factors,
                                   want_left, want_right)
    if getattr(f, "shard_rrlu", False) and not want_factors:
        return f.update_pivots_sharded(rows, cols, maxrank, reltol, abstol, leftorth)
    if getattr(f, "device_gather", False):  # sharded evaluation, Pi gathered in HBM over RCCL
        return f.update_pivots_gathered(rows, cols, maxrank, reltol, abstol, leftorth, want_factors,
                                        want_left, want_right)
    if not hasattr(f, "h"):
        return _update_pivots_generic(f, rows, cols, maxrank, reltol, abstol, leftorth, want_factors,
                                      want_left, want_right)
    ctx = f.ctx
    rows = np.ascontiguousarray(rows, np.int32)
    cols = np.ascontiguousarray(cols, np.int32)
    m, nl = rows.shape
    n, nr = cols.shape
    mr = int(max(min(int(maxrank), m, n), 0))
    rowidx = np.zeros(max(mr, 1), np.int64)
    colidx = np.zeros(max(mr, 1), np.int64)
    pe = np.zeros(mr + 1)
    npv = C.c_int64()
    mx = C.c_double()
    # (large factor buffers recycled from replaced site tensors: every value read back is written)
    left = _POOL.take(m * mr) if (want_factors and want_left) else None
    right = _POOL.take(mr * n) if (want_factors and want_right) else None
    ctx.check(ctx.lib.tci_update_pivots_h(ctx.h, f.h, _lib.ptr(rows), m, nl, _lib.ptr(cols), n, nr,
                                          int(min(maxrank, INT64_MAX)), float(reltol), float(abstol),
                                          int(bool(leftorth)), int(bool(want_factors)), _lib.ptr(rowidx),
                                          _lib.ptr(colidx), _lib.ptr(pe), C.byref(npv), C.byref(mx),
                                          _lib.ptr(left), _lib.ptr(right)))
    k = npv.value
    res = {"rowidx": rowidx[:k].copy(), "colidx": colidx[:k].copy(), "pivoterrors": pe[: k + 1].copy(),
           "maxabs": mx.value, "npivot": k}
    if left is not None:
        res["left"] = left[: m * k].reshape((m, k), order="F")
    if right is not None:
        res["right"] = right[: k * n].reshape((k, n), order="F")
    return res


def _update_pivots_c128(f, rows, cols, maxrank, reltol, abstol, leftorth, want_factors,
                        want_left, want_right):
    """The 2-site update of a ComplexF64 evaluator: Pi, max|Pi|, complex rrLU and MatrixLUCI
    factors in one device call (tci_update_pivots_c128_h)."""
    ctx = f.ctx
    rows = np.ascontiguousarray(rows, np.int32)
    cols = np.ascontiguousarray(cols, np.int32)
    m, nl = rows.shape
    n, nr = cols.shape
    mr = int(max(min(int(maxrank), m, n), 0))
    rowidx = np.zeros(max(mr, 1), np.int64)
    colidx = np.zeros(max(mr, 1), np.int64)
    pe = np.zeros(mr + 1)
    npv = C.c_int64()
    mx = C.c_double()
    left = np.zeros(max(m * mr, 1), np.complex128) if (want_factors and want_left) else None
    right = np.zeros(max(mr * n, 1), np.complex128) if (want_factors and want_right) else None
    ctx.check(ctx.lib.tci_update_pivots_c128_h(ctx.h, f.f.h, f.coeff.real, f.coeff.imag, _lib.ptr(rows), m, nl,
                                               _lib.ptr(cols), n, nr, int(min(maxrank, INT64_MAX)),
                                               float(reltol), float(abstol), int(bool(leftorth)),
                                               int(bool(want_factors)), _lib.ptr(rowidx), _lib.ptr(colidx),
                                               _lib.ptr(pe), C.byref(npv), C.byref(mx), _lib.ptr(left),
                                               _lib.ptr(right)))
    k = npv.value
    res = {"rowidx": rowidx[:k].copy(), "colidx": colidx[:k].copy(), "pivoterrors": pe[: k + 1].copy(),
           "maxabs": mx.value, "npivot": k}
    if left is not None:
        res["left"] = left[: m * k].reshape((m, k), order="F")
    if right is not None:
        res["right"] = right[: k * n].reshape((k, n), order="F")
    return res


def _update_pivots_generic(f, rows, cols, maxrank, reltol, abstol, leftorth, want_factors,
                           want_left, want_right):
    ctx = _ctx_of(f)
    Pi, mx = f.pi(np.asarray(rows, np.int32), np.asarray(cols, np.int32), 0)
    cplx = np.iscomplexobj(Pi)  # MatrixLUCI{ComplexF64}
    dt = np.complex128 if cplx else np.float64
    Pi = np.asfortranarray(Pi, dt)
    m, n = Pi.shape
    mr = int(max(min(int(maxrank), m, n), 0))
    rowidx = np.zeros(max(mr, 1), np.int64)
    colidx = np.zeros(max(mr, 1), np.int64)
    pe = np.zeros(mr + 1)
    npv = C.c_int64()
    left = np.zeros(max(m * mr, 1), dt) if (want_factors and want_left) else None
    right = np.zeros(max(mr * n, 1), dt) if (want_factors and want_right) else None
    ctx.check((ctx.lib.tci_luci_c128_h if cplx else ctx.lib.tci_luci_h)(ctx.h, _lib.ptr(Pi), m, n, max(m, 1), int(min(maxrank, INT64_MAX)),
                                 float(reltol), float(abstol), int(bool(leftorth)), _lib.ptr(rowidx),
                                 _lib.ptr(colidx), _lib.ptr(pe), _lib.ptr(left), _lib.ptr(right),
                                 C.byref(npv)))
    k = npv.value
    res = {"rowidx": rowidx[:k].copy(), "colidx": colidx[:k].copy(), "pivoterrors": pe[: k + 1].copy(),
           "maxabs": mx, "npivot": k}
    if left is not None:
        res["left"] = left[: m * k].reshape((m, k), order="F")
    if right is not None:
        res["right"] = right[: k * n].reshape((k, n), order="F")
    return res


def _sitetensor_generic(f, Ib, Jb, Inext, solve):
    Pi1, mx = f.pi(np.asarray(Ib, np.int32), np.asarray(Jb, np.int32), 1)
    if not solve:
        return None, mx
    if Inext is None:
        return np.asfortranarray(Pi1), mx
    P, _ = f.pi(np.asarray(Inext, np.int32), np.asarray(Jb, np.int32), 0)
    r = P.shape[0]
    if P.shape[0] != P.shape[1]:
        raise RuntimeError("Pivot matrix is not square!")
    R = Pi1.shape[0]
    ctx = _ctx_of(f)
    if np.iscomplexobj(Pi1) or np.iscomplexobj(P):
        T = np.zeros(max(R * r, 1), np.complex128)
        ctx.check(ctx.lib.tci_sitetensor_solve_c128_h(ctx.h, _lib.ptr(np.asfortranarray(P, np.complex128)), r,
                                                      _lib.ptr(np.asfortranarray(Pi1, np.complex128)), R,
                                                      _lib.ptr(T)))
        return T[: R * r].reshape((R, r), order="F"), mx
    T = np.zeros(max(R * r, 1))
    ctx.check(ctx.lib.tci_sitetensor_solve_h(ctx.h, _lib.ptr(np.asfortranarray(P, np.float64)), r,
                                             _lib.ptr(np.asfortranarray(Pi1, np.float64)), R, _lib.ptr(T)))
    return T[: R * r].reshape((R, r), order="F"), mx


def sitetensor_device(f, Ib, Jb, Inext, solve=True):
    """T = Pi1 * P^-1 (tensorci2.jl:599-629) on the device; returns (T or None, max|Pi1|)."""
    if getattr(f, "is_complex", False):
        Pi1, mx = f.pi(Ib, Jb, 1, want_values=solve)
        if not solve or Inext is None:
            return (np.asfortranarray(Pi1) if solve else None), mx
        P, _ = f.pi(Inext, Jb, 0)
        if P.shape[0] != P.shape[1]:
            raise RuntimeError("Pivot matrix is not square!")
        r, R = P.shape[0], Pi1.shape[0]
        T = np.zeros(max(R * r, 1), np.complex128)
        ctx = f.ctx
        ctx.check(ctx.lib.tci_sitetensor_solve_c128_h(ctx.h, _lib.ptr(np.asfortranarray(P)), r,
                                                      _lib.ptr(np.asfortranarray(Pi1)), R, _lib.ptr(T)))
        return T[: R * r].reshape((R, r), order="F"), mx
    if getattr(f, "device_gather", False):
        return f.sitetensor_gathered(Ib, Jb, Inext, solve)
    if not hasattr(f, "h"):
        return _sitetensor_generic(f, Ib, Jb, Inext, solve)
    ctx = f.ctx
    Ib = np.ascontiguousarray(Ib, np.int32)
    Jb = np.ascontiguousarray(Jb, np.int32)
    nI, wI = Ib.shape
    nJ, wJ = Jb.shape
    d = f.localdims[wI]
    R = nI * d
    mx = C.c_double()
    if Inext is None:
        T = _POOL.take(R * nJ) if solve else None  # (written in full by the device copy)
        nxt, nn = None, 0
    else:
        Inext = np.ascontiguousarray(Inext, np.int32)
        nn = len(Inext)
        T = _POOL.take(R * nn) if solve else None
        nxt = Inext
    if not solve:
        # only max|Pi1| is observable: evaluate Pi1 on the device, no solve, no copy back
        I = Ib
        out_mx = _batch_maxabs(f, I, Jb, 1)
        return None, out_mx
    ctx.check(ctx.lib.tci_sitetensor_h(ctx.h, f.h, _lib.ptr(Ib), nI, wI, _lib.ptr(Jb), nJ, wJ, _lib.ptr(nxt),
                                       nn, _lib.ptr(T), C.byref(mx)))
    cols = nJ if Inext is None else nn
    return T[: R * cols].reshape((R, cols), order="F"), mx.value


def _batch_maxabs(f, I, J, M):
    if not hasattr(f, "h"):
        return f.pi(I, J, M)[1]
    ctx = f.ctx
    m, nl = I.shape
    n, nr = J.shape
    D = f.localdims[nl] if M == 1 else 1
    mx = C.c_double()
    scratch = _scratch(ctx, m * D * n)
    ctx.check(ctx.lib.tci_batcheval_d(ctx.h, f.h, _lib.ptr(I), m, nl, _lib.ptr(J), n, nr, M, scratch,
                                      max(m * D, 1), C.byref(mx)))
    return mx.value


class _Scratch:
    """Per-context device scratch for Pi evaluations whose values are not needed (only max|.|)."""

    def __init__(self, ctx, nelem):
        self.ctx = ctx
        self.size = max(int(nelem * 1.5), 1024)
        p = C.c_void_p()
        ctx.check(ctx.lib.tci_malloc_d(ctx.h, C.byref(p), self.size * 8))
        self.ptr = p
        ctx.own(self)

    def release(self):
        if self.ptr and self.ctx.alive:
            self.ctx.lib.tci_free_d(self.ctx.h, self.ptr)
        self.ptr = None


def _scratch(ctx, nelem):
    cur = getattr(ctx, "_scratch", None)
    if cur is None or cur.ptr is None or cur.size < nelem:
        if cur is not None:
            cur.release()
        cur = ctx._scratch = _Scratch(ctx, nelem)
    return cur.ptr


def crossinterpolate2(f, localdims=None, initialpivots=None, **kwargs):
    """crossinterpolate2(Float64, f, localdims, initialpivots; kwargs...) (tensorci2.jl:1313-1323).
    Returns (tci, ranks, errors)."""
    if localdims is None:
        localdims = f.localdims
    tci = TensorCI2.from_function(f, localdims, initialpivots)
    ranks, errors = tci.optimize(f, **kwargs)
    return tci, ranks, errors


def optfirstpivot(f, localdims, firstpivot=None, maxsweep=1000):
    """optfirstpivot (util.jl:260-298). Within one leg only that leg changes, so the d candidate
    values of a leg are evaluated in one device call and then scanned in the reference's order
    (strict '>' against the running best, which is exactly the sequential loop)."""
    L = len(localdims)
    pivot = list(firstpivot) if firstpivot is not None else [1] * L
    valf = abs(f.points([pivot])[0])
    for _ in range(maxsweep):
        valf_prev = valf
        for i in range(L):
            cand = np.tile(np.asarray(pivot, np.int32), (localdims[i], 1))
            cand[:, i] = np.arange(1, localdims[i] + 1)
            vals = np.abs(f.points(cand))
            for d in range(localdims[i]):
                if vals[d] > valf:
                    valf = vals[d]
                    pivot[i] = d + 1
        if valf_prev == valf:
            break
    return [int(x) for x in pivot]
