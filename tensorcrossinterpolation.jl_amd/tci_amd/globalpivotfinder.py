"""Global pivot search -- mirror of src/globalpivotfinder.jl.

DefaultGlobalPivotFinder (globalpivotfinder.jl:145-265): nsearch random points; from each, a line
search along every leg records the point of largest |f(x) - tt(x)|; points whose error exceeds
abstol * tolmarginglobalsearch become global pivots (at most maxnglobalpivot). All nsearch *
sum(localdims) candidate points are evaluated in ONE device batch call, and the tensor train on
the host in one batched contraction. The reference draws points from Julia's default_rng; numpy's
generator is used here, so this search matches the reference only statistically.

Multi-GPU ("the global pivot search (independent random starts) also shards"): with a
ShardedBatchEvaluator the nsearch starts are drawn once on rank 0 and broadcast, each rank runs the
line searches of the starts s with s % world == rank on its own GPU (f and the tensor train), and
the per-start results (largest error and its point) are all-gathered, so every rank adds the same
pivots in start order -- the same list one process finds from the same starts.
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
        comm = getattr(f, "comm", None)
        world = comm.world if comm is not None else 1
        starts = np.stack([rng.integers(1, d + 1, size=self.nsearch) for d in localdims], axis=1)
        if world > 1:  # rank 0's starts everywhere
            starts = comm.allgather_flat(starts.ravel().astype(np.float64))[: starts.size].reshape(starts.shape)
            starts = starts.astype(np.int64)
        mine = [s for s in range(self.nsearch) if s % world == (comm.rank if world > 1 else 0)]
        per = sum(localdims)
        # all line-search candidates of this rank's starts: start s, leg p, value v -> start with
        # leg p set to v
        cands = []
        for s in mine:
            for p in range(L):
                for v in range(1, localdims[p] + 1):
                    x = starts[s].copy()
                    x[p] = v
                    cands.append(x)
        X = np.asarray(cands, np.int32).reshape(-1, L)
        ctx = getattr(f, "ctx", None) or getattr(getattr(f, "local", None), "ctx", None)
        ev = f.local if world > 1 else f  # sharded: this rank's GPU evaluates its own starts
        err = np.abs(ev.points(X) - tci.evaluate_many(X, ctx=ctx)) if len(X) else np.zeros(0)
        # per start: (best error, index of its point in the start's line-search set) or (0, -1)
        res = np.zeros((self.nsearch, 2))
        res[:, 1] = -1
        for t, s in enumerate(mine):
            e = err[t * per:(t + 1) * per]
            best_i, best = -1, 0.0
            for i, v in enumerate(e):  # strict '>' from best_error = 0.0 (globalpivotfinder.jl:239)
                if v > best:
                    best, best_i = v, i
            res[s] = (best, best_i)
        if world > 1:
            allr = comm.allgather_flat(res.ravel()).reshape(world, self.nsearch, 2)
            res = np.array([allr[s % world, s] for s in range(self.nsearch)])
        found = []
        for s in range(self.nsearch):
            best, best_i = res[s, 0], int(res[s, 1])
            if best_i >= 0 and best > abstol * self.tolmarginglobalsearch:
                p, v = 0, best_i
                while v >= localdims[p]:
                    v -= localdims[p]
                    p += 1
                x = starts[s].copy()
                x[p] = v + 1
                found.append([int(t) for t in x])
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
