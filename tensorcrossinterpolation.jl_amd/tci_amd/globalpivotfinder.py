"""Global pivot search -- mirror of src/globalpivotfinder.jl.

DefaultGlobalPivotFinder (globalpivotfinder.jl:145-265): nsearch random points; from each, a line
search along every leg records the point of largest |f(x) - tt(x)|; points whose error exceeds
abstol * tolmarginglobalsearch become global pivots (at most maxnglobalpivot). All nsearch *
sum(localdims) candidate points are evaluated in ONE device batch call, and the tensor train on
the host in one batched contraction. The reference draws points from Julia's default_rng; numpy's
generator is used here, so this search matches the reference only statistically.
"""
import numpy as np


class AbstractGlobalPivotFinder:
    """abstract type AbstractGlobalPivotFinder (globalpivotfinder.jl:84): callable as
    finder(tci, f, abstol; verbosity, rng) -> list of MultiIndex."""

    nsearch = 1

    def __call__(self, tci, f, abstol, verbosity=0, rng=None):
        raise NotImplementedError(f"find_global_pivots not implemented for {type(self).__name__}")


class DefaultGlobalPivotFinder(AbstractGlobalPivotFinder):
    def __init__(self, nsearch=5, maxnglobalpivot=5, tolmarginglobalsearch=10.0):
        self.nsearch = int(nsearch)
        self.maxnglobalpivot = int(maxnglobalpivot)
        self.tolmarginglobalsearch = float(tolmarginglobalsearch)

    def __call__(self, tci, f, abstol, verbosity=0, rng=None):
        if self.nsearch <= 0:
            return []
        rng = rng if rng is not None else np.random.default_rng()
        localdims = tci.localdims
        L = len(localdims)
        starts = np.stack([rng.integers(1, d + 1, size=self.nsearch) for d in localdims], axis=1)
        # all line-search candidates: for start s, leg p, value v -> start with leg p set to v
        cands = []
        for s in range(self.nsearch):
            for p in range(L):
                for v in range(1, localdims[p] + 1):
                    x = starts[s].copy()
                    x[p] = v
                    cands.append(x)
        X = np.asarray(cands, np.int32)
        ctx = getattr(f, "ctx", None) or getattr(getattr(f, "local", None), "ctx", None)
        err = np.abs(f.points(X) - tci.evaluate_many(X, ctx=ctx))
        found = []
        off = 0
        per = sum(localdims)
        for s in range(self.nsearch):
            e = err[off:off + per]
            best_i, best = -1, 0.0
            for i, v in enumerate(e):  # strict '>' from best_error = 0.0 (globalpivotfinder.jl:239)
                if v > best:
                    best, best_i = v, i
            if best_i >= 0 and best > abstol * self.tolmarginglobalsearch:
                found.append(X[off + best_i].tolist())
            off += per
        if len(found) > self.maxnglobalpivot:
            found = found[: self.maxnglobalpivot]
        if verbosity > 0:
            print(f"Found {len(found)} global pivots")
        return found


class FixedGlobalPivotFinder(AbstractGlobalPivotFinder):
    """Deterministic finder that injects a fixed list once (the plugin route SURVEY §8(b) names
    for reproducible parity runs; compare test_tensorci2.jl:105-118)."""

    def __init__(self, pivots):
        self.pivots = [list(map(int, p)) for p in pivots]
        self.nsearch = 1

    def __call__(self, tci, f, abstol, verbosity=0, rng=None):
        out, self.pivots = self.pivots, []
        return out
