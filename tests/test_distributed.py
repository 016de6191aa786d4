"""Multi-process tests of the sharded batch evaluation (tci_amd/distributed.py).

CPU tests: world_size 2 (and 3) over gloo, with a test-only evaluator backed by the oracle, so
the product's sharding, NaN-propagating maxsample reduction and column all-gather are checked
against the single-process evaluation. GPU test: two ranks sharing cuda:0 (gloo for the
exchange) run crossinterpolate2 through ShardedBatchEvaluator and must reproduce the
single-process run bitwise. The parent process never touches the GPU (children are spawned).
"""
import json
import os
import socket
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, os.path.join(ROOT, "tensorcrossinterpolation.jl_amd"))

from tci_amd.distributed import Comm, ShardedBatchEvaluator, column_blocks  # noqa: E402


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_column_blocks():
    for n in (0, 1, 5, 8, 37, 1000):
        for world in (1, 2, 3, 8):
            b = column_blocks(n, world)
            assert len(b) == world and b[0][0] == 0 and b[-1][1] == n
            assert all(b[r][1] == b[r + 1][0] for r in range(world - 1))
            w = [j1 - j0 for j0, j1 in b]
            assert max(w) - min(w) <= 1


class OracleEvaluator:
    """Test-only stand-in for a rank's GPUBatchEvaluator: the oracle's batch evaluation."""

    def __init__(self, kind, params, localdims):
        import oracle_lib as O

        self.O, self.kind, self.params, self.localdims = O, kind, params, list(localdims)

    def pi(self, I, J, M=0):
        out, mx = self.O.batcheval(self.kind, self.params, self.localdims, I, J, M)
        return out.reshape((-1, len(J)), order="F"), mx

    def points(self, X):
        X = np.asarray(X, np.int32).reshape(-1, len(self.localdims))
        return self.pi(np.zeros((1, 0), np.int32), X)[0][0, :].copy()


class ZeroTT:
    """Test-only stand-in for a TensorCI2 in the global search: tt(x) = 0, so |f - tt| = |f|."""

    def __init__(self, localdims):
        self.localdims = list(localdims)

    def evaluate_many(self, X, ctx=None):
        return np.zeros(len(X))


def _cpu_worker(rank, world, port, outdir):
    import torch.distributed as dist

    sys.path.insert(0, HERE)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        rng = np.random.default_rng(7)
        res = {}
        # Lorentzian (integer-exact) and a table with a NaN in the last column block
        ld = [6] * 6
        table = rng.random(int(np.prod(ld)))
        for name, kind, params in (("lorentz", 1, [1.0]), ("table", 2, table.tolist())):
            for M in (0, 1):
                nl = 2
                nr = 6 - nl - M
                I = rng.integers(1, 7, (23, nl)).astype(np.int32)
                J = rng.integers(1, 7, (31, nr)).astype(np.int32)
                f = ShardedBatchEvaluator(OracleEvaluator(kind, params, ld), Comm(device="cpu"))
                full, mx = f.pi(I, J, M)
                ref, rmx = OracleEvaluator(kind, params, ld).pi(I, J, M)
                res[f"{name}{M}"] = bool(np.array_equal(full, ref)) and (mx == rmx)
        # NaN in a column only the last rank evaluates: every rank must see maxabs = NaN
        t2 = table.copy()
        J = np.array([[1, 1, 1, 1]] * 9 + [[6, 6, 6, 6]], np.int32)
        I = np.array([[1, 1]] * 4, np.int32)
        t2[np.ravel_multi_index((0, 0, 5, 5, 5, 5), ld, order="F")] = np.nan
        f = ShardedBatchEvaluator(OracleEvaluator(2, t2.tolist(), ld), Comm(device="cpu"))
        _, mx = f.pi(I, J, 0)
        res["nan"] = bool(np.isnan(mx))
        # more ranks than columns: empty blocks
        f = ShardedBatchEvaluator(OracleEvaluator(1, [1.0], ld), Comm(device="cpu"))
        full, mx = f.pi(I, J[:1], 0)
        ref, rmx = OracleEvaluator(1, [1.0], ld).pi(I, J[:1], 0)
        res["empty_blocks"] = bool(np.array_equal(full, ref)) and mx == rmx
        pts = rng.integers(1, 7, (13, 6)).astype(np.int32)
        got = f.points(pts)
        ref = OracleEvaluator(1, [1.0], ld).pi(np.zeros((1, 0), np.int32), pts, 0)[0][0]
        res["points"] = bool(np.array_equal(got, ref))
        with open(os.path.join(outdir, f"rank{rank}.json"), "w") as fh:
            json.dump(res, fh)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_batcheval_gloo(tmp_path, world):
    import torch.multiprocessing as mp

    mp.spawn(_cpu_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    for r in range(world):
        res = json.load(open(tmp_path / f"rank{r}.json"))
        assert all(res.values()), (r, res)


def _gpu_worker(rank, world, port, outdir, shard_rrlu=False):
    import torch.distributed as dist

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        import tci_amd as T

        ctx = T.context(0)
        local = T.lorentz([8] * 6, ctx=ctx)
        fs = ShardedBatchEvaluator(local, Comm(device="cpu"), shard_rrlu=shard_rrlu)
        kw = dict(tolerance=1e-10, maxiter=8, nsearchglobalpivot=0)
        tci, ranks, errors = T.crossinterpolate2(fs, [8] * 6, **kw)
        ref, rranks, rerrors = T.crossinterpolate2(local, [8] * 6, **kw)
        q = T.quantics_osc(16, ctx=ctx)
        p0 = T.optfirstpivot(q, [2] * 16)
        qs = ShardedBatchEvaluator(q, Comm(device="cpu"), shard_rrlu=shard_rrlu)
        t2, r2, e2 = T.crossinterpolate2(qs, [2] * 16, [p0], tolerance=1e-8, maxiter=6, nsearchglobalpivot=0)
        t2r, r2r, e2r = T.crossinterpolate2(q, [2] * 16, [p0], tolerance=1e-8, maxiter=6, nsearchglobalpivot=0)
        # with the default global pivot search, starts split over the ranks (same seed as one process)
        kwg = dict(tolerance=1e-10, maxiter=8, nsearchglobalpivot=5)
        tg, rg, eg = T.crossinterpolate2(fs, [8] * 6, rng=np.random.default_rng(3), **kwg)
        tgr, rgr, egr = T.crossinterpolate2(local, [8] * 6, rng=np.random.default_rng(3), **kwg)
        res = {
            "global_search": rg == rgr and list(eg) == list(egr)
                             and all(np.array_equal(a, b) for a, b in zip(tg.Iset, tgr.Iset)),
            "ranks": ranks == rranks, "errors": list(errors) == list(rerrors),
            "isets": all(np.array_equal(a, b) for a, b in zip(tci.Iset, ref.Iset)),
            "jsets": all(np.array_equal(a, b) for a, b in zip(tci.Jset, ref.Jset)),
            "qosc": r2 == r2r and list(e2) == list(e2r),
            "linkdims": tci.linkdims(),
        }
        with open(os.path.join(outdir, f"rank{rank}.json"), "w") as fh:
            json.dump(res, fh)
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("shard_rrlu", [False, True])
def test_sharded_tci2_two_ranks_one_gpu(tmp_path, shard_rrlu):
    """shard_rrlu=False: Pi all-gathered, replicated rrLU; True: Pi stays sharded on the device and
    the column-sharded rrLU factorises it across the ranks (host exchange: two ranks share cuda:0)."""
    import torch.multiprocessing as mp

    mp.spawn(_gpu_worker, args=(2, _free_port(), str(tmp_path), shard_rrlu), nprocs=2, join=True)
    res = [json.load(open(tmp_path / f"rank{r}.json")) for r in range(2)]
    for r in res:
        assert r["ranks"] and r["errors"] and r["isets"] and r["jsets"] and r["qosc"] and r["global_search"], r
    assert res[0]["linkdims"] == res[1]["linkdims"]


def _gpu_fail_worker(rank, world, port, outdir):
    import torch.distributed as dist

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        import tci_amd as T

        ctx = T.context(0)
        local = T.lorentz([8] * 6, ctx=ctx)
        fs = ShardedBatchEvaluator(local, Comm(device="cpu"), shard_rrlu=True)
        kw = dict(tolerance=1e-10, maxiter=8, nsearchglobalpivot=0)
        lib = ctx.lib
        real = lib.tci_batcheval_da
        calls = [0]

        def failing(*a):  # the last rank's deferred evaluation fails from its third call on
            calls[0] += 1
            return 1 if calls[0] >= 3 else real(*a)

        res = {}
        if rank == world - 1:
            lib.tci_batcheval_da = failing
        try:
            T.crossinterpolate2(fs, [8] * 6, **kw)
            res["raised"] = None
        except T.TCIError as e:
            res["raised"] = "own:" + str(e)
        except RuntimeError as e:
            res["raised"] = "other:" + str(e)
        finally:
            lib.tci_batcheval_da = real
        res["calls"] = calls[0]
        # the group and the device path are still usable afterwards
        tci, ranks, errors = T.crossinterpolate2(fs, [8] * 6, **kw)
        ref, rranks, rerrors = T.crossinterpolate2(local, [8] * 6, **kw)
        res["after"] = ranks == rranks and list(errors) == list(rerrors)
        with open(os.path.join(outdir, f"rank{rank}.json"), "w") as fh:
            json.dump(res, fh)
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.timeout(240)
def test_sharded_deferred_eval_failure_two_ranks_one_gpu(tmp_path):
    """with shard_rrlu the block is evaluated by tci_batcheval_da and max|Pi| reduced only
    after the sharded rrLU; a rank whose evaluation fails still takes part in the factorisation and
    then raises, and every other rank raises with it in the same reduction -- nobody is left inside
    an exchange, and the group works afterwards."""
    import torch.multiprocessing as mp

    mp.spawn(_gpu_fail_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    for r in range(2):
        res = json.load(open(tmp_path / f"rank{r}.json"))
        want = "own:" if r == 1 else "other:"
        assert res["raised"] and res["raised"].startswith(want) and res["after"], (r, res)


# ------------------------------------------------------------------ column-sharded rrLU protocol
def _shard_worker(rank, world, port, outdir, fused=False):
    import torch.distributed as dist

    sys.path.insert(0, HERE)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        import oracle_lib as O
        from sharded_protocol import sharded_rrlu

        comm = Comm(device="cpu")
        res = {}
        rng = np.random.default_rng(11)
        cases = {
            "random": (rng.random((37, 29)), {}),
            # integer Lorentzian values: exact ties across column blocks (tie order by position)
            "ties": (1.0 / (1.0 + np.add.outer(np.arange(40) % 5, np.arange(33) % 4) ** 2), {}),
            "rightorth": (rng.random((25, 31)), {"leftorth": False}),
            "maxrank": (rng.random((30, 30)), {"maxrank": 7}),
            "lowrank_stop": (rng.random((40, 3)) @ rng.random((3, 26)), {"reltol": 1e-10}),
            "wide_few_cols": (rng.random((12, 4)), {}),  # world 3: ranks with 1-2 columns
        }
        for name, (A, kw) in cases.items():
            m, n = A.shape
            j0, j1 = column_blocks(n, world)[rank]
            npv, err, rp, cp, L, U = sharded_rrlu(A[:, j0:j1], m, n, j0, comm.allgather_flat,
                                                  comm.allreduce_max_u64, fused=fused, **kw)
            U = comm.allreduce_sum(U)
            ref = O.OracleLU(A, maxrank=kw.get("maxrank", min(m, n)), reltol=kw.get("reltol", 1e-14),
                             leftorthogonal=kw.get("leftorth", True))
            res[name] = bool(npv == ref.npivot and np.array_equal(rp, ref.rowpermutation)
                             and np.array_equal(cp, ref.colpermutation) and np.array_equal(L, ref.L)
                             and np.array_equal(U, ref.U) and (err == ref.error or (np.isnan(err) and np.isnan(ref.error))))
        with open(os.path.join(outdir, f"rank{rank}.json"), "w") as fh:
            json.dump(res, fh)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("fused", [False, True])
def test_sharded_rrlu_protocol_gloo(tmp_path, world, fused):
    """The column-sharded rrLU protocol (local argmax, all-gather of the candidates, the winning
    column from its owner through a uint64 max -- or, fused, one all-gather of candidates with
    their columns -- the same commit on every rank) reproduces the unsharded oracle bit for bit
    (tests/sharded_protocol.py)."""
    import torch.multiprocessing as mp

    mp.spawn(_shard_worker, args=(world, _free_port(), str(tmp_path), fused), nprocs=world, join=True)
    for r in range(world):
        res = json.load(open(tmp_path / f"rank{r}.json"))
        assert all(res.values()), (r, res)


def _search_worker(rank, world, port, outdir):
    import torch.distributed as dist

    sys.path.insert(0, HERE)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        from tci_amd.globalpivotfinder import DefaultGlobalPivotFinder

        ld = [5, 7, 4, 6, 3]
        res = {}
        for nsearch in (1, 5, 9):
            finder = DefaultGlobalPivotFinder(nsearch=nsearch, maxnglobalpivot=5)
            fs = ShardedBatchEvaluator(OracleEvaluator(1, [1.0], ld), Comm(device="cpu"))
            # rank 0's generator decides the starts; the single-process run uses the same seed
            got = finder(ZeroTT(ld), fs, 1e-6, rng=np.random.default_rng(100 + nsearch if rank == 0 else 7))
            ref = finder(ZeroTT(ld), OracleEvaluator(1, [1.0], ld), 1e-6, rng=np.random.default_rng(100 + nsearch))
            res[f"n{nsearch}"] = got == ref and len(ref) == min(nsearch, 5)
        with open(os.path.join(outdir, f"rank{rank}.json"), "w") as fh:
            json.dump(res, fh)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_global_search_gloo(tmp_path, world):
    """The global pivot search with its starts split over the ranks finds the same pivots, in the
    same order, as one process from the same starts (globalpivotfinder.jl:219-252)."""
    import torch.multiprocessing as mp

    mp.spawn(_search_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    for r in range(world):
        res = json.load(open(tmp_path / f"rank{r}.json"))
        assert all(res.values()), (r, res)


class _RaisesOnLastRank(OracleEvaluator):
    """Test-only evaluator whose f fails on the last rank's column block only (a user's f raising
    for some inputs, as a HostFunctionEvaluator's callback may)."""

    def __init__(self, rank, world, *a):
        super().__init__(*a)
        self.fail = rank == world - 1

    def pi(self, I, J, M=0):
        if self.fail:
            raise ValueError("f failed on this rank's columns")
        return super().pi(I, J, M)


def _fail_worker(rank, world, port, outdir):
    import torch.distributed as dist

    sys.path.insert(0, HERE)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        ld = [6] * 6
        I = np.array([[1, 2]] * 5, np.int32)
        J = np.array([[1, 2, 3, 4]] * 11, np.int32)
        f = ShardedBatchEvaluator(_RaisesOnLastRank(rank, world, 1, [1.0], ld), Comm(device="cpu"))
        res = {}
        try:
            f.pi(I, J, 0)
            res["raised"] = None
        except ValueError as e:
            res["raised"] = "own:" + str(e)
        except RuntimeError as e:
            res["raised"] = "other:" + str(e)
        # the group is still usable afterwards (nobody is left inside a collective)
        ok = ShardedBatchEvaluator(OracleEvaluator(1, [1.0], ld), Comm(device="cpu"))
        full, _ = ok.pi(I, J, 0)
        res["after"] = bool(np.array_equal(full, OracleEvaluator(1, [1.0], ld).pi(I, J, 0)[0]))
        with open(os.path.join(outdir, f"rank{rank}.json"), "w") as fh:
            json.dump(res, fh)
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(120)
@pytest.mark.parametrize("world", [2, 3])
def test_sharded_failure_raises_on_every_rank(tmp_path, world):
    """a batch evaluation failing on one rank only must raise on every rank (the flag
    travels in the max|Pi| reduction before any data collective), not leave the others blocked."""
    import torch.multiprocessing as mp

    mp.spawn(_fail_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    for r in range(world):
        res = json.load(open(tmp_path / f"rank{r}.json"))
        want = "own:" if r == world - 1 else "other:"
        assert res["raised"] and res["raised"].startswith(want) and res["after"], (r, res)
