"""Column-sharded rrLU on the device (tci_rrlu_sharded_d), through the C ABI:
bitwise against the unsharded oracle (permutations, npivot, lu.error, pivot errors, L, U).

* one rank (no exchange) in-process: the sharded driver's passes + ghost column + commit;
* 2 and 3 ranks sharing cuda:0 with the host exchange hook (gloo) -- RCCL refuses two ranks on one
  device, so this is how the multi-rank device path is checked on a one-GPU box;
* one rank through an RCCL communicator (tci_comm_*: unique id over gloo, ncclAllGather on the
  context stream): the RCCL data path of bench.py --gpus N.
The parent process never touches the GPU in the multi-process tests (children are spawned).
Reference: /root/reference/src/matrixlu.jl:46-87 (submatrixargmax), :295-322 (addpivot!),
:346-396 (_optimizerrlu!).
"""
import json
import os
import socket
import sys

import numpy as np
import pytest

import oracle_lib as O

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
T = pytest.importorskip("tci_amd")
from tci_amd.distributed import Comm, DeviceComm, HostExchange, column_blocks, rrlu_sharded, rrlu_sharded_factors  # noqa: E402


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _cases():
    rng = np.random.default_rng(5)
    return {
        "random_1000x900_r100": (O.fill_uniform(1000 * 900, 3).reshape((1000, 900), order="F"), dict(maxrank=100)),
        "ties_lorentz_600x500": (1.0 / (1.0 + np.add.outer(np.arange(600) % 7, np.arange(500) % 5) ** 2),
                                 dict(maxrank=60)),
        "rightorth_700x800_r50": (rng.random((700, 800)), dict(maxrank=50, leftorth=False)),
        "lowrank_stop": (rng.random((400, 12)) @ rng.random((12, 300)), dict(reltol=1e-10)),
        "tall_8300x120_r40": (O.fill_uniform(8300 * 120, 4).reshape((8300, 120), order="F"), dict(maxrank=40)),
    }


def _run_rank(ctx, A, rank, world, kw, comm=None, exchange=None):
    m, n = A.shape
    j0, j1 = column_blocks(n, world)[rank]
    nloc = j1 - j0
    loc = T.DeviceMatrix(m, nloc + 1, ctx=ctx)
    loc.upload(np.hstack([A[:, j0:j1], np.zeros((m, 1))]))
    out = rrlu_sharded(loc, m, n, j0, nloc, comm=comm, exchange=exchange, nranks=world,
                       maxrank=kw.get("maxrank"), reltol=kw.get("reltol", 1e-14),
                       leftorthogonal=kw.get("leftorth", True))
    loc.free()
    return out


def _check(A, kw, out, L, U):
    npv, err, rp, cp, pe = out
    ref = O.OracleLU(A, maxrank=kw.get("maxrank", min(A.shape)), reltol=kw.get("reltol", 1e-14),
                     leftorthogonal=kw.get("leftorth", True))
    res = {"npivot": npv == ref.npivot,
           "rowperm": bool(np.array_equal(rp - 1, ref.rowpermutation)),
           "colperm": bool(np.array_equal(cp - 1, ref.colpermutation)),
           "error": bool(err == ref.error),
           "pivoterrors": bool(np.array_equal(pe, ref.pivoterrors)),
           "L": bool(np.array_equal(L, ref.L)), "U": bool(np.array_equal(U, ref.U))}
    return res


@pytest.fixture(scope="module")
def ctx():
    c = T.Context(0)
    yield c
    c.close()


@pytest.mark.parametrize("name", list(_cases()))
@pytest.mark.parametrize("shadow,epochs", [(1, 0), (0, 0), (1, 3)])
def test_sharded_one_rank_bitwise(ctx, name, shadow, epochs):
    """epochs 3: the two-level epoch (refresh passes, EXT passes, the deep write-back) in the
    sharded driver; 0: the by-shape default (1 at these sizes)."""
    A, kw = _cases()[name]
    ctx.check(ctx.lib.tci_set_rrlu_shadow(ctx.h, shadow))
    ctx.check(ctx.lib.tci_set_rrlu_epochs(ctx.h, epochs))
    try:
        out = _run_rank(ctx, A, 0, 1, kw)
        L, U = rrlu_sharded_factors(ctx, A.shape[0], A.shape[1], out[0])
    finally:
        ctx.check(ctx.lib.tci_set_rrlu_shadow(ctx.h, 1))
        ctx.check(ctx.lib.tci_set_rrlu_epochs(ctx.h, 0))
    res = _check(A, kw, out, L, U)
    assert all(res.values()), res


def _multi_worker(rank, world, port, outdir, mode, epochs=0, exmode=0):
    import torch.distributed as dist

    sys.path.insert(0, HERE)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        ctx = T.Context(0)
        ctx.check(ctx.lib.tci_set_rrlu_epochs(ctx.h, epochs))
        ctx.check(ctx.lib.tci_set_shard_exchange(ctx.h, exmode))
        host = Comm(device="cpu")
        comm = exchange = None
        if mode == "rccl":
            comm = DeviceComm(ctx, host)
        else:
            exchange = HostExchange(ctx, host)
        res = {}
        for name, (A, kw) in _cases().items():
            out = _run_rank(ctx, A, rank, world, kw, comm=comm, exchange=exchange)
            L, U = rrlu_sharded_factors(ctx, A.shape[0], A.shape[1], out[0], host_comm=host)
            res[name] = _check(A, kw, out, L, U)
            # the exchange that ran: fused (2) by size at these shapes unless forced
            res[name]["exchange"] = ctx.lib.tci_last_shard_exchange(ctx.h) == (exmode or 2)
        if comm is not None:
            comm.close()
        ctx.close()
        with open(os.path.join(outdir, f"rank{rank}.json"), "w") as fh:
            json.dump(res, fh)
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("world,mode,epochs,exmode", [
    (2, "host", 0, 1), (2, "host", 0, 2), (3, "host", 0, 1), (3, "host", 0, 0), (1, "rccl", 0, 1),
    (1, "rccl", 0, 2), (2, "host", 3, 1), (2, "host", 3, 2), (1, "rccl", 3, 0)])
def test_sharded_multi_rank_bitwise(tmp_path, world, mode, epochs, exmode):
    """epochs 3: the two-level epoch across ranks (the ghost column carries every exact-pending y).
    exmode: the per-pivot exchange -- 1 two collectives (record all-gather + column max-broadcast),
    2 the fused all-gather of record + own candidate column, 0 by size (fused here)."""
    import torch.multiprocessing as mp

    mp.spawn(_multi_worker, args=(world, _free_port(), str(tmp_path), mode, epochs, exmode), nprocs=world,
             join=True)
    for r in range(world):
        res = json.load(open(tmp_path / f"rank{r}.json"))
        bad = {k: v for k, v in res.items() if not all(v.values())}
        assert not bad, (r, bad)


def _mismatch_worker(rank, world, port, outdir):
    import torch.distributed as dist

    sys.path.insert(0, HERE)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        ctx = T.Context(0)
        ctx.check(ctx.lib.tci_set_shard_exchange(ctx.h, 1 + rank % 2))  # rank 0 two collectives, rank 1 fused
        exchange = HostExchange(ctx, Comm(device="cpu"))
        A, kw = _cases()["random_1000x900_r100"]
        res = {}
        try:
            _run_rank(ctx, A, rank, world, kw, exchange=exchange)
            res["raised"] = None
        except T.TCIArgumentError as e:
            res["raised"] = str(e)
        # agreeing again, the same ranks factorise bitwise
        ctx.check(ctx.lib.tci_set_shard_exchange(ctx.h, 0))
        out = _run_rank(ctx, A, rank, world, kw, exchange=exchange)
        L, U = rrlu_sharded_factors(ctx, A.shape[0], A.shape[1], out[0], host_comm=Comm(device="cpu"))
        res["after"] = all(_check(A, kw, out, L, U).values())
        ctx.close()
        with open(os.path.join(outdir, f"rank{rank}.json"), "w") as fh:
            json.dump(res, fh)
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(200)
def test_sharded_exchange_forms_must_agree(tmp_path):
    """the exchange form follows each rank's own setting; ranks that disagree fail
    together with TCI_ERR_ARG (one agreement reduction per factorisation) instead of issuing
    collectives of different kinds and counts."""
    import torch.multiprocessing as mp

    mp.spawn(_mismatch_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    for r in range(2):
        res = json.load(open(tmp_path / f"rank{r}.json"))
        assert res["raised"] and "exchange forms" in res["raised"] and res["after"], (r, res)


def _gather_worker(rank, world, port, outdir):
    import torch.distributed as dist

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        from tci_amd.distributed import ShardedBatchEvaluator
        ctx = T.Context(0)
        host = Comm(device="cpu")
        dcomm = DeviceComm(ctx, host)
        res = {}
        local = T.lorentz([8] * 6, ctx=ctx)
        kw = dict(tolerance=1e-10, maxiter=8, nsearchglobalpivot=0)
        ref, rranks, rerrors = T.crossinterpolate2(local, [8] * 6, **kw)
        for shard in (False, True):
            fs = ShardedBatchEvaluator(local, host, shard_rrlu=shard, device_comm=dcomm)
            assert fs.device_gather
            tci, ranks, errors = T.crossinterpolate2(fs, [8] * 6, **kw)
            res[f"shard{int(shard)}"] = bool(
                ranks == rranks and list(errors) == list(rerrors)
                and all(np.array_equal(a, b) for a, b in zip(tci.Iset, ref.Iset))
                and all(np.array_equal(a, b) for a, b in zip(tci.Jset, ref.Jset))
                and all(np.allclose(a, b, rtol=1e-12, atol=1e-14) for a, b in zip(tci.sitetensors, ref.sitetensors)))
        # the gathered Pi itself, bitwise the local evaluation
        fs = ShardedBatchEvaluator(local, host, device_comm=dcomm)
        rng = np.random.default_rng(4)
        I = rng.integers(1, 9, (37, 2)).astype(np.int32)
        J = rng.integers(1, 9, (53, 4)).astype(np.int32)
        view, gmx = fs.pi_device(I, J, 0)
        buf = np.empty(view.ld * view.n)
        ctx.check(ctx.lib.tci_memcpy_d2h(ctx.h, buf.ctypes.data, view.ptr, buf.nbytes))
        got = buf.reshape((view.ld, view.n), order="F")[:view.m, :]
        want, wmx = local.pi(I, J, 0)
        res["pi_device"] = bool(np.array_equal(got, want) and gmx == wmx)
        dcomm.close()
        ctx.close()
        with open(os.path.join(outdir, f"rank{rank}.json"), "w") as fh:
            json.dump(res, fh)
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_sharded_device_gather_one_rccl_rank(tmp_path):
    """The sharded evaluation's factor / site-tensor path with Pi gathered in HBM over RCCL
    (ShardedBatchEvaluator.pi_device -> tci_luci_inplace_d / tci_sitetensor_solve_d; VERDICT r2
    missing #2): a whole TCI2 run equals the single-process one (ranks, errors, index sets bitwise;
    site tensors to 1e-12), with the replicated and the column-sharded rrLU. One RCCL rank (a
    one-GPU box); N > 1 is the same code with more slots in the all-gather."""
    import torch.multiprocessing as mp

    mp.spawn(_gather_worker, args=(1, _free_port(), str(tmp_path)), nprocs=1, join=True)
    res = json.load(open(tmp_path / "rank0.json"))
    assert all(res.values()), res


def _metric_worker(rank, world, port, outdir):
    """The metric matrix (8192^2 U[0,1), seed 0: bench.py's) column-sharded over `world` ranks with
    the host exchange and the two-level epoch forced (epochs = 3: refreshes, EXT passes, the deep
    write-back, the ghost column carrying every exact-pending y); rank 0 checks against the oracle."""
    import torch.distributed as dist

    sys.path.insert(0, HERE)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        ctx = T.Context(0)
        ctx.check(ctx.lib.tci_set_rrlu_epochs(ctx.h, 3))
        host = Comm(device="cpu")
        m = n = 8192
        A = O.fill_uniform(m * n, seed=0).reshape((m, n), order="F")
        kw = dict(maxrank=256)
        out = _run_rank(ctx, A, rank, world, kw, exchange=HostExchange(ctx, host))
        L, U = rrlu_sharded_factors(ctx, m, n, out[0], host_comm=host)
        res = _check(A, kw, out, L, U) if rank == 0 else {"skipped": True}
        res["fused_exchange"] = ctx.lib.tci_last_shard_exchange(ctx.h) == 2
        ctx.close()
        with open(os.path.join(outdir, f"rank{rank}.json"), "w") as fh:
            json.dump(res, fh)
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(600)
def test_sharded_two_ranks_metric_epochs3(tmp_path):
    """two ranks (host exchange, sharing cuda:0) at the metric size 8192^2, r = 256, with
    epochs = 3 -- bitwise the unsharded oracle (permutations, npivot, lu.error, pivot errors, L, U)."""
    import torch.multiprocessing as mp

    mp.spawn(_metric_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    res = json.load(open(tmp_path / "rank0.json"))
    assert all(res.values()), res
