"""Single-rank timing of the column-sharded rrLU (tci_rrlu_sharded_d over a one-rank RCCL
communicator) against the unsharded device rrLU on the same matrix: the per-pivot cost of the
gather / all-gather / commit sequence. python scripts/sharded_timing.py"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tensorcrossinterpolation.jl_amd"))
import tci_amd as T  # noqa: E402
from tci_amd.distributed import DeviceComm, rrlu_sharded  # noqa: E402

ctx = T.Context(0)
dc = DeviceComm(ctx)
for m, r in ((8192, 256), (16384, 256)):
    n = m
    A0 = T.DeviceMatrix(m, n + 1, ctx=ctx)
    A0.fill_uniform(seed=0)
    W = T.DeviceMatrix(m, n + 1, ctx=ctx)
    res = {}
    for mode in ("unsharded", "sharded"):
        ts = []
        for _ in range(3):
            W.copy_from(A0)
            ctx.synchronize()
            t0 = time.perf_counter()
            if mode == "sharded":
                rrlu_sharded(W, m, n, 0, n, comm=dc, maxrank=r)
            else:
                Wv = T.distributed._DevView(ctx, W.ptr, m, n, W.ld)
                T.rrlu_inplace_device(Wv, maxrank=r, want_perms=False)
            ctx.synchronize()
            ts.append(time.perf_counter() - t0)
        res[mode] = min(ts) * 1e3
    print(f"{m}^2 r={r}: unsharded {res['unsharded']:.2f} ms, sharded(1 rank) {res['sharded']:.2f} ms, "
          f"overhead {(res['sharded'] - res['unsharded']) / r * 1e3:.1f} us/pivot", flush=True)
    A0.free()
    W.free()
dc.close()
