"""Multi-GPU sharding of the batch evaluation.

One process per GPU (torch.distributed: "nccl" is RCCL over xGMI on ROCm, "gloo" for host
buffers and CPU tests). Pi assembly is embarrassingly parallel over elements, so the columns of
Jcomb are split into contiguous blocks, one per rank: each rank evaluates Pi[:, j0:j1] on its own
GPU (column-major, so a block is contiguous), maxsample is all-reduced with Julia's
NaN-propagating max (updatemaxsample!, tensorci2.jl:636-638 / util.jl:34-43), and the blocks are
all-gathered only where a replicated Pi is needed (the replicated rrLU that follows in
updatepivots!, tensorci2.jl:842-868). Every rank then holds bitwise the same Pi, so the
replicated factorisations agree exactly and all ranks keep identical TCI2 state.

`ShardedBatchEvaluator` wraps any evaluator with the `pi(I, J, M) -> (matrix, maxabs)` method of
`GPUBatchEvaluator` and is itself such an evaluator, so `crossinterpolate2` takes it unchanged.
"""
import ctypes as C
import math

import numpy as np


def column_blocks(n, world):
    """Balanced contiguous blocks [(j0, j1)] of n columns over `world` ranks (rank order)."""
    base, rem = divmod(int(n), int(world))
    out, j = [], 0
    for r in range(world):
        w = base + (1 if r < rem else 0)
        out.append((j, j + w))
        j += w
    return out


class Comm:
    """torch.distributed facade for the two collectives the sharded path needs.

    device: the torch device of the collective buffers ("cpu" for gloo; "cuda:<local rank>" for
    nccl, i.e. RCCL on ROCm). Data is exchanged as float64 tensors.
    """

    def __init__(self, group=None, device="cpu"):
        import torch
        import torch.distributed as dist

        self.torch = torch
        self.dist = dist
        self.group = group
        self.device = device
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)

    def allreduce_maxabs(self, x, error=None):
        """max over ranks with Julia's NaN propagation (any NaN -> NaN). `error`: an exception this
        rank's local work raised; the flag travels in the same reduction, so when any rank failed
        EVERY rank raises here together (the failing one its own error) instead of the others
        blocking in the next collective."""
        torch = self.torch
        isn = error is None and math.isnan(x)
        val = -math.inf if (isn or error is not None) else float(x)
        t = torch.tensor([val, 1.0 if isn else 0.0, 1.0 if error is not None else 0.0], dtype=torch.float64,
                         device=self.device)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX, group=self.group)
        if t[2].item() > 0:
            if error is not None:
                raise error
            raise RuntimeError("batch evaluation failed on another rank")
        return math.nan if t[1].item() > 0 else float(t[0].item())

    def allgather_columns(self, block, blocks, rows):
        """Concatenate the ranks' column blocks (rows x (j1 - j0), Fortran order) into the full
        rows x n matrix, identical on every rank."""
        torch = self.torch
        wmax = max(j1 - j0 for j0, j1 in blocks)
        n = blocks[-1][1]
        buf = torch.zeros(rows * max(wmax, 1), dtype=torch.float64, device=self.device)
        if block.size:
            buf[: block.size] = torch.from_numpy(np.asarray(block, np.float64).ravel(order="F")).to(self.device)
        out = torch.empty(self.world * buf.numel(), dtype=torch.float64, device=self.device)
        self.dist.all_gather_into_tensor(out, buf, group=self.group)
        out = out.cpu().numpy().reshape(self.world, -1)
        full = np.empty((rows, n), order="F")
        for r, (j0, j1) in enumerate(blocks):
            if j1 > j0:
                full[:, j0:j1] = out[r, : rows * (j1 - j0)].reshape((rows, j1 - j0), order="F")
        return full

    def barrier(self):
        self.dist.barrier(group=self.group)

    def broadcast_bytes(self, arr, src=0):
        """uint8 array from rank `src` to every rank."""
        torch = self.torch
        t = torch.from_numpy(np.ascontiguousarray(arr, np.uint8).copy()).to(self.device)
        self.dist.broadcast(t, src=src, group=self.group)
        return t.cpu().numpy()

    def allgather_flat(self, buf):
        """float64 vectors of equal length from every rank, concatenated in rank order."""
        torch = self.torch
        t = torch.from_numpy(np.ascontiguousarray(buf, np.float64)).to(self.device)
        out = torch.empty(self.world * t.numel(), dtype=torch.float64, device=self.device)
        self.dist.all_gather_into_tensor(out, t, group=self.group)
        return out.cpu().numpy()

    def allreduce_max_u64(self, words):
        """element-wise max over the ranks of uint64 vectors (bit patterns; equal lengths)."""
        w = np.ascontiguousarray(words, np.uint64)
        allb = self.allgather_flat(w.view(np.float64)).reshape(self.world, -1)
        return np.ascontiguousarray(allb).view(np.uint64).max(axis=0)

    def allreduce_sum(self, a):
        torch = self.torch
        a = np.asarray(a, np.float64)
        t = torch.from_numpy(np.asfortranarray(a).ravel(order="F").copy()).to(self.device)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.SUM, group=self.group)
        return t.cpu().numpy().reshape(a.shape, order="F")


class ShardedBatchEvaluator:
    """A BatchEvaluator{Float64} whose batch evaluation is split over the ranks of `comm` by
    column blocks of Jset; each rank's block runs on its own GPU through `local` (a
    GPUBatchEvaluator on that rank's device).

    shard_rrlu: the 2-site update keeps Pi sharded on the devices -- each rank evaluates its column
    block into HBM and the column-sharded rrLU (tci_rrlu_sharded_d) factorises it across the ranks,
    exchanging one candidate record per pivot over `device_comm` (a DeviceComm: RCCL) or, without
    one, over the host group (HostExchange). Pi never leaves the devices and is never replicated.
    Without shard_rrlu (or when the MatrixLUCI factors are needed) Pi is all-gathered and factorised
    replicated, as before."""

    def __init__(self, local, comm, shard_rrlu=False, device_comm=None):
        self.local = local
        self.comm = comm
        self.localdims = list(local.localdims)
        self.L = len(self.localdims)
        self.name = f"sharded({getattr(local, 'name', 'f')})"
        self.shard_rrlu = bool(shard_rrlu)
        self.device_comm = device_comm
        self._exchange = None
        self._buf = None

    @property
    def ctx(self):
        return self.local.ctx

    def exchange(self):
        if self.device_comm is None and self._exchange is None:
            self._exchange = HostExchange(self.local.ctx, self.comm)
        return self._exchange

    def local_block_device(self, I, J, M=0, defer_max=False):
        """This rank's block of Pi evaluated into HBM, as an m x (nloc + 1) device matrix (the last
        column is the sharded rrLU's scratch), plus (j0, j1) and the global max|Pi|.

        defer_max (catalog integrands): the block is evaluated with tci_batcheval_da -- the index
        tables uploaded asynchronously, max|Pi| folded into a device word, no host synchronisation
        -- and the third result is a callable that reads the word and reduces it over the ranks
        (with any local evaluation error, so that a failure raises on every rank together). The
        caller runs the collective work that follows first (the sharded rrLU, which synchronises at
        its end), then calls it: one host synchronisation per bond."""
        from . import _lib

        ctx = self.local.ctx
        if defer_max and getattr(self.local, "kind", None) not in (None, 10):  # 10: TCI_F_HOST
            return self._local_block_deferred(I, J, M)
        I = np.ascontiguousarray(np.asarray(I, np.int32))
        J = np.ascontiguousarray(np.asarray(J, np.int32))
        m, nl = I.shape
        D = self.localdims[nl] if M == 1 else 1
        j0, j1 = self.block(len(J))
        nloc = j1 - j0
        rows = m * D
        ld = max(16, (rows + 15) // 16 * 16)
        need = ld * (nloc + 1)
        if self._buf is None or self._buf.size < need:
            if self._buf is not None:
                self._buf.free()
            self._buf = _DevBuf(ctx, int(need * 1.25) + 1024)
        view = _DevView(ctx, self._buf.ptr, rows, nloc + 1, ld)
        mx, err = 0.0, None
        if nloc > 0 and rows > 0:
            Jl = np.ascontiguousarray(J[j0:j1])
            m_ = C.c_double()
            try:
                ctx.check(ctx.lib.tci_batcheval_d(ctx.h, self.local.h, _lib.ptr(I), m, nl, _lib.ptr(Jl), nloc,
                                                  Jl.shape[1], M, view.ptr, ld, C.byref(m_)))
                mx = m_.value
            except Exception as e:  # raised on every rank by the reduction (no rank left waiting)
                err = e
        return view, (j0, j1), self.comm.allreduce_maxabs(mx, err)

    def _local_block_deferred(self, I, J, M):
        from . import _lib

        ctx = self.local.ctx
        I = np.ascontiguousarray(np.asarray(I, np.int32))
        J = np.ascontiguousarray(np.asarray(J, np.int32))
        m, nl = I.shape
        D = self.localdims[nl] if M == 1 else 1
        j0, j1 = self.block(len(J))
        nloc = j1 - j0
        rows = m * D
        ld = max(16, (rows + 15) // 16 * 16)
        need = ld * (nloc + 1)
        if self._buf is None or self._buf.size < need:
            if self._buf is not None:
                self._buf.free()
            self._buf = _DevBuf(ctx, int(need * 1.25) + 1024)
        if getattr(self, "_maxword", None) is None:
            self._maxword = _DevBuf(ctx, 1)
        view = _DevView(ctx, self._buf.ptr, rows, nloc + 1, ld)
        err = None
        try:
            # the max word zeroed stream-ordered (no host synchronisation), then the block
            ctx.check(ctx.lib.tci_memset_d(ctx.h, self._maxword.ptr, 0, 8))
            if nloc > 0 and rows > 0:
                Jl = np.ascontiguousarray(J[j0:j1])
                ctx.check(ctx.lib.tci_batcheval_da(ctx.h, self.local.h, _lib.ptr(I), m, nl, _lib.ptr(Jl), nloc,
                                                   Jl.shape[1], M, view.ptr, ld, self._maxword.ptr))
        except Exception as e:  # raised on every rank by the deferred reduction
            err = e

        def reduce_max():
            nonlocal err
            mx = 0.0
            if err is None and nloc > 0 and rows > 0:
                try:  # a failed read-back also reaches the reduction: no rank is left waiting in it
                    bits = np.zeros(1, np.uint64)
                    ctx.check(ctx.lib.tci_memcpy_d2h(ctx.h, _lib.ptr(bits), self._maxword.ptr, 8))
                    mx = float(bits.view(np.float64)[0])
                except Exception as e:
                    err = e
            return self.comm.allreduce_maxabs(mx, err)

        return view, (j0, j1), reduce_max

    @property
    def device_gather(self):
        """A replicated Pi can be assembled in HBM by RCCL (no host staging)."""
        return self.device_comm is not None

    def pi_device(self, I, J, M=0, slot=0):
        """Full (|I| * D) x |J| Pi replicated in HBM on every rank, with no host staging (SURVEY 8(e)
        C1): each rank evaluates its block of w = ceil(|J| / N) columns into its slot of a padded
        ld x (N w) buffer and ONE ncclAllGather (in place, on the context stream) fills the other
        slots; the first |J| columns are Pi. Returns (view, max|Pi| over the ranks). slot selects
        one of two buffers (Pi1 and P of a site tensor)."""
        from . import _lib

        ctx = self.local.ctx
        I = np.ascontiguousarray(np.asarray(I, np.int32))
        J = np.ascontiguousarray(np.asarray(J, np.int32))
        m, nl = I.shape
        n, nr = J.shape
        D = self.localdims[nl] if M == 1 else 1
        rows = m * D
        N, r = self.comm.world, self.comm.rank
        w = max(1, -(-n // N))
        ld = max(16, (rows + 15) // 16 * 16)
        need = ld * w * N
        bufs = self.__dict__.setdefault("_gbufs", [None, None])
        if bufs[slot] is None or bufs[slot].size < need:
            if bufs[slot] is not None:
                bufs[slot].free()
            bufs[slot] = _DevBuf(ctx, int(need * 1.25) + 1024)
        base = bufs[slot].ptr.value
        j0, j1 = min(r * w, n), min((r + 1) * w, n)
        mx, err = 0.0, None
        if j1 > j0 and rows > 0:
            Jl = np.ascontiguousarray(J[j0:j1])
            m_ = C.c_double()
            try:
                ctx.check(ctx.lib.tci_batcheval_d(ctx.h, self.local.h, _lib.ptr(I), m, nl, _lib.ptr(Jl), j1 - j0,
                                                  nr, M, C.c_void_p(base + 8 * ld * w * r), ld, C.byref(m_)))
                mx = m_.value
            except Exception as e:  # e.g. a HostFunctionEvaluator's f raising on this rank only
                err = e
        # agree on success (and max|Pi|) over the host group BEFORE the RCCL all-gather, so a
        # failure on one rank raises on every rank instead of leaving the others in ncclAllGather
        gmx = self.comm.allreduce_maxabs(mx, err)
        if rows > 0:
            self.device_comm.allgather(C.c_void_p(base + 8 * ld * w * r), C.c_void_p(base), 8 * ld * w)
        return _DevView(ctx, C.c_void_p(base), rows, n, ld), gmx

    def update_pivots_gathered(self, rows, cols, maxrank, reltol, abstol, leftorth, want_factors,
                               want_left=True, want_right=True):
        """updatepivots! with the factors (first half-sweep, sweep1site!): Pi all-gathered in HBM
        over RCCL, MatrixLUCI on this rank's GPU (tci_luci_inplace_d); every rank computes the same
        bits. Same result dict as tensorci2.update_pivots_device."""
        from . import _lib

        ctx = self.local.ctx
        view, gmx = self.pi_device(rows, cols, 0)
        m, n = view.m, view.n
        mr = int(max(min(int(maxrank), m, n), 0))
        rowidx = np.zeros(max(mr, 1), np.int64)
        colidx = np.zeros(max(mr, 1), np.int64)
        pe = np.zeros(mr + 1)
        npv = C.c_int64()
        left = np.zeros(max(m * mr, 1)) if (want_factors and want_left) else None
        right = np.zeros(max(mr * n, 1)) if (want_factors and want_right) else None
        ctx.check(ctx.lib.tci_luci_inplace_d(ctx.h, view.ptr, m, n, view.ld, int(min(maxrank, 2 ** 62)),
                                             float(reltol), float(abstol), int(bool(leftorth)), _lib.ptr(rowidx),
                                             _lib.ptr(colidx), _lib.ptr(pe), _lib.ptr(left), _lib.ptr(right),
                                             C.byref(npv)))
        k = npv.value
        res = {"rowidx": rowidx[:k].copy(), "colidx": colidx[:k].copy(), "pivoterrors": pe[: k + 1].copy(),
               "maxabs": gmx, "npivot": k}
        if left is not None:
            res["left"] = left[: m * k].reshape((m, k), order="F")
        if right is not None:
            res["right"] = right[: k * n].reshape((k, n), order="F")
        return res

    def sitetensor_gathered(self, Ib, Jb, Inext, solve=True):
        """setsitetensor!'s T = Pi1 P^-1 (tensorci2.jl:599-629) with Pi1 and P all-gathered in HBM
        and the solve on this rank's GPU (tci_sitetensor_solve_d); only T comes to the host."""
        ctx = self.local.ctx
        if not solve:
            _, _, gmx = self.pi_local(Ib, Jb, 1)
            return None, gmx
        v1, gmx = self.pi_device(Ib, Jb, 1, slot=0)
        R, r = v1.m, v1.n
        if Inext is None:  # the last site: T = Pi1
            if R * r == 0:
                return np.zeros((R, r), order="F"), gmx
            buf = np.empty(v1.ld * r)
            ctx.check(ctx.lib.tci_memcpy_d2h(ctx.h, C.c_void_p(buf.ctypes.data), v1.ptr, buf.nbytes))
            return np.asfortranarray(buf.reshape((v1.ld, r), order="F")[:R, :]), gmx
        vp_, _ = self.pi_device(Inext, Jb, 0, slot=1)
        if vp_.m != vp_.n:
            raise RuntimeError("Pivot matrix is not square!")
        if R == 0 or r == 0:
            return np.zeros((R, r), order="F"), gmx
        from .matrixlu import DeviceMatrix
        P = DeviceMatrix(r, r, ctx=ctx, ld=r)
        Pi1 = DeviceMatrix(R, r, ctx=ctx, ld=R)
        Tm = DeviceMatrix(R, r, ctx=ctx, ld=R)
        try:
            ctx.check(ctx.lib.tci_memcpy2d_d2d(ctx.h, P.ptr, 8 * r, vp_.ptr, 8 * vp_.ld, 8 * r, r))
            ctx.check(ctx.lib.tci_memcpy2d_d2d(ctx.h, Pi1.ptr, 8 * R, v1.ptr, 8 * v1.ld, 8 * R, r))
            ctx.check(ctx.lib.tci_sitetensor_solve_d(ctx.h, P.ptr, r, Pi1.ptr, R, Tm.ptr))
            return Tm.to_host().copy(order="F"), gmx
        finally:
            for x in (P, Pi1, Tm):
                x.free()

    def update_pivots_sharded(self, rows, cols, maxrank, reltol, abstol, leftorth):
        """updatepivots!'s :full search with Pi sharded on the devices: returns the dict of
        tensorci2.update_pivots_device (pivot positions, pivot errors, max|Pi|; no factors)."""
        rows = np.asarray(rows, np.int32)
        cols = np.asarray(cols, np.int32)
        # catalog integrands: the block evaluated without a host synchronisation, max|Pi| reduced
        # after the factorisation (whose end synchronises anyway); a rank whose evaluation failed
        # still takes part in the sharded rrLU (on whatever its block holds) and then raises with
        # every other rank in the reduction -- no rank is left waiting in an exchange
        view, (j0, j1), gmx = self.local_block_device(rows, cols, 0, defer_max=True)
        m, n = len(rows), len(cols)
        npv, err, rp, cp, pe = rrlu_sharded(view, m, n, j0, j1 - j0, comm=self.device_comm,
                                            exchange=None if self.device_comm is not None else self.exchange(),
                                            maxrank=min(int(maxrank), m, n), reltol=reltol, abstol=abstol,
                                            leftorthogonal=leftorth)
        if callable(gmx):
            gmx = gmx()
        return {"rowidx": rp[:npv].copy(), "colidx": cp[:npv].copy(), "pivoterrors": pe.copy(), "maxabs": gmx,
                "npivot": npv}

    def block(self, n):
        """This rank's column range of an n-column Pi."""
        return column_blocks(n, self.comm.world)[self.comm.rank]

    def pi_local(self, I, J, M=0):
        """This rank's block Pi[:, j0:j1] and the global max|Pi| (no gather)."""
        I = np.ascontiguousarray(np.asarray(I, np.int32))
        J = np.ascontiguousarray(np.asarray(J, np.int32))
        D = self.localdims[I.shape[1]] if M == 1 else 1
        j0, j1 = self.block(len(J))
        blk, mx, err = np.zeros((I.shape[0] * D, 0), order="F"), 0.0, None
        if j1 > j0:
            try:
                blk, mx = self.local.pi(I, J[j0:j1], M)
            except Exception as e:  # raised on every rank by the reduction below
                err = e
        return (j0, j1), blk, self.comm.allreduce_maxabs(mx, err)

    def pi(self, I, J, M=0):
        """Full (|I| * D) x |J| Pi on every rank, and max|Pi|."""
        I = np.asarray(I, np.int32)
        J = np.asarray(J, np.int32)
        D = self.localdims[I.shape[1]] if M == 1 else 1
        _, blk, gmx = self.pi_local(I, J, M)
        full = self.comm.allgather_columns(blk, column_blocks(len(J), self.comm.world), I.shape[0] * D)
        return full, gmx

    def points(self, X):
        X = np.asarray(X, np.int32).reshape(-1, self.L)
        out, _ = self.pi(np.zeros((1, 0), np.int32), X)  # the points become the columns
        return out[0, :].copy()

    def __call__(self, x, Jset=None, M=None):
        if Jset is not None:
            return self.batch(x, Jset, M)
        return float(self.points(np.asarray(x).reshape(1, -1))[0])

    def batch(self, Iset, Jset, M):
        M = int(M)
        if len(Iset) * len(Jset) == 0:
            return np.zeros((0,) * (M + 2))
        nl, nr = len(Iset[0]), len(Jset[0])
        if nl + M + nr != self.L:
            raise ValueError("Invalid number of central indices")
        I = np.asarray(Iset, np.int32).reshape(len(Iset), nl)
        J = np.asarray(Jset, np.int32).reshape(len(Jset), nr)
        out, _ = self.pi(I, J, M)
        return out.reshape((len(Iset),) + tuple(self.localdims[nl:nl + M]) + (len(Jset),), order="F")


# ------------------------------------------------------------------ device-resident data path
class _DevBuf:
    """Raw device allocation owned by a context (float64 elements)."""

    def __init__(self, ctx, nelem):
        self.ctx, self.size = ctx, int(nelem)
        p = C.c_void_p()
        ctx.check(ctx.lib.tci_malloc_d(ctx.h, C.byref(p), self.size * 8))
        self.ptr = p
        ctx.own(self)

    def free(self):
        if self.ptr and self.ctx.alive:
            self.ctx.lib.tci_free_d(self.ctx.h, self.ptr)
        self.ptr = None

    release = free


class _DevView:
    """m x n column-major view (ld) of device memory, DeviceMatrix-like."""

    def __init__(self, ctx, ptr, m, n, ld):
        self.ctx, self.ptr, self.m, self.n, self.ld = ctx, ptr, int(m), int(n), int(ld)


class DeviceComm:
    """An RCCL communicator inside libtci_hip.so (tci_comm_*), bound to a context's device and
    stream: collectives on device buffers, enqueued on the context stream -- no host staging.
    The 128-byte unique id goes from rank 0 to the others over `comm` (a `Comm`, i.e. the
    torch.distributed host group)."""

    def __init__(self, ctx, comm=None):
        from . import _lib

        self.ctx = ctx
        self.rank, self.world = (comm.rank, comm.world) if comm is not None else (0, 1)
        lib = ctx.lib
        nbytes = C.c_int64()
        ctx.check(lib.tci_comm_unique_id(None, C.byref(nbytes)))
        uid = np.zeros(nbytes.value, np.uint8)
        if self.rank == 0:
            ctx.check(lib.tci_comm_unique_id(_lib.ptr(uid), None))
        if comm is not None:
            uid = comm.broadcast_bytes(uid)
        h = C.c_void_p()
        ctx.check(lib.tci_comm_create(ctx.h, self.world, self.rank, _lib.ptr(uid), C.byref(h)))
        self.h = h
        ctx.own(self)

    def allgather(self, d_send, d_recv, nbytes):
        self.ctx.check(self.ctx.lib.tci_comm_allgather_d(self.h, d_send, d_recv, int(nbytes)))

    def release(self):
        if getattr(self, "h", None) and self.ctx.alive:
            self.ctx.lib.tci_comm_destroy(self.h)
        self.h = None

    close = release


class HostExchange:
    """The tci_exchange_fn hook over a host `Comm` (gloo): device -> host, collective, host ->
    device. For ranks that cannot form an RCCL communicator (several ranks on one GPU, CPU-side
    transports); correct everywhere, slower than DeviceComm.

    Failures are collective: every rank always enters the host collective, with an ok flag next to
    its data, and every rank reports failure when any rank's flag is down -- so a copy that fails
    on one rank cannot leave the others waiting in the next exchange."""

    def __init__(self, ctx, comm):
        from . import _lib

        self.ctx, self.comm = ctx, comm
        self._lib = _lib

        def fn(user, op, d_send, d_recv, count):
            count = int(count)
            ok = 1.0
            buf = np.zeros(count, np.uint64)
            try:
                ctx.check(ctx.lib.tci_memcpy_d2h(ctx.h, _lib.ptr(buf), d_send, buf.nbytes))
            except Exception:
                ok = 0.0
            try:
                if op == 0:  # all-gather of the words, with the flag as one extra word per rank
                    allb = comm.allgather_flat(np.concatenate([buf.view(np.float64), [ok]]))
                    allb = allb.reshape(comm.world, count + 1)
                    if not np.all(allb[:, count] == 1.0):
                        return 1
                    out = np.ascontiguousarray(allb[:, :count]).ravel()
                else:  # element-wise uint64 max: all-gather and reduce (bit patterns, no float compare)
                    allb = comm.allgather_flat(np.concatenate([buf.view(np.float64), [ok]]))
                    allb = allb.reshape(comm.world, count + 1)
                    if not np.all(allb[:, count] == 1.0):
                        return 1
                    out = np.ascontiguousarray(allb[:, :count]).view(np.uint64).max(axis=0)
                ctx.check(ctx.lib.tci_memcpy_h2d(ctx.h, d_recv, _lib.ptr(np.ascontiguousarray(out)), out.nbytes))
                return 0
            except Exception:
                return 1

        self.fn = _lib.EXCHANGE_FN(fn)  # keep a reference for the library's lifetime of the call


def rrlu_sharded(local, m, n, c0, nloc, comm=None, exchange=None, nranks=1, maxrank=None, reltol=1e-14,
                 abstol=0.0, leftorthogonal=True):
    """Column-sharded rrlu! over the ranks (tci_rrlu_sharded_d): `local` is this rank's DeviceMatrix
    holding global columns [c0, c0 + nloc) as its columns 0..nloc-1 plus one scratch column (so
    local.n == nloc + 1). comm: a DeviceComm (RCCL) or exchange: a HostExchange; neither for one
    rank. Returns (npivot, error, rowperm, colperm, pivoterrors), identical on every rank and
    bitwise those of rrlu on the full matrix (1-based permutations)."""
    from . import _lib

    ctx = local.ctx
    if local.n != nloc + 1 or local.m != m:
        raise ValueError("rrlu_sharded: the local matrix must be m x (nloc + 1)")
    mr = min(m, n) if maxrank is None else int(maxrank)
    rowperm = np.zeros(max(m, 1), np.int64)
    colperm = np.zeros(max(n, 1), np.int64)
    pe = np.zeros(max(min(mr, m, n), 0) + 1)
    npv, err = C.c_int64(), C.c_double()
    world = comm.world if comm is not None else (exchange.comm.world if exchange is not None else nranks)
    ctx.check(ctx.lib.tci_rrlu_sharded_d(ctx.h, comm.h if comm is not None else None,
                                         exchange.fn if exchange is not None else None, None, int(world),
                                         local.ptr, m, nloc, local.ld, c0, n, int(min(mr, 2 ** 62)),
                                         float(reltol), float(abstol), int(bool(leftorthogonal)),
                                         _lib.ptr(rowperm), _lib.ptr(colperm), C.byref(npv), C.byref(err),
                                         _lib.ptr(pe)))
    k = npv.value
    return k, err.value, rowperm[:m], colperm[:n], pe[: k + 1]


def rrlu_sharded_factors(ctx, m, n, npivot, host_comm=None):
    """L (m x np) and U (np x n) of the last rrlu_sharded on `ctx`, position order. U's columns are
    combined over the ranks with `host_comm` (each rank fills only its own columns)."""
    from . import _lib

    L = np.zeros((m, npivot), order="F")
    U = np.zeros((npivot, n), order="F")
    if npivot == 0:
        return L, U
    st = ctx.lib.tci_rrlu_sharded_factors_h(ctx.h, L.ctypes.data_as(C.c_void_p), U.ctypes.data_as(C.c_void_p),
                                            npivot)
    if host_comm is not None and host_comm.world > 1:
        # the NaN checks (matrixlu.jl:376-381) see only this rank's columns of U: agree on the
        # status first, so that every rank raises together instead of one rank raising while the
        # others wait in the sum below
        codes = host_comm.allgather_flat(np.array([float(st)]))
        bad = [int(c) for c in codes if c != 0]
        if bad:
            if st == 0:
                st = bad[0]
                from . import _lib
                raise _lib.TCIError(st, "lu.U contains NaNs" if st == _lib.TCI_ERR_NAN else
                                    f"rrlu_sharded_factors failed on another rank (code {st})")
            ctx.check(st)
        U = host_comm.allreduce_sum(U)
    else:
        ctx.check(st)
    return L, U
