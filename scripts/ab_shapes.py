"""rrLU epoch-schedule A/B over shapes (device-resident, pass pipeline as the library picks it):
for every (m, n, r) and every (nb, epochs) setting, the median of `reps` factorisations
(copy + rrlu_inplace_device, like bench.py's rrlu_configs). One JSON line per (shape, setting).

  python scripts/ab_shapes.py [--reps 5] [--set nb,epochs ...] [--shape MxNxR ...]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tensorcrossinterpolation.jl_amd"))

import tci_amd as T  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--set", action="append", default=None, help="nb,epochs")
    ap.add_argument("--shape", action="append", default=None, help="MxNxR")
    a = ap.parse_args()
    sets = [tuple(int(x) for x in s.split(",")) for s in (a.set or ["10,3", "10,2", "10,1", "11,1", "8,1", "12,1"])]
    shapes = [tuple(int(x) for x in s.split("x")) for s in (a.shape or ["2048x2048x256", "4096x4096x256",
                                                                        "8192x8192x256", "16384x16384x256"])]
    ctx = T.context()
    for (m, n, r) in shapes:
        A = T.DeviceMatrix(m, n, ctx=ctx)
        A.fill_uniform(seed=0)
        W = T.DeviceMatrix(m, n, ctx=ctx)
        for (nb, ep) in sets:
            ctx.check(ctx.lib.tci_set_rrlu_flush(ctx.h, nb))
            ctx.check(ctx.lib.tci_set_rrlu_epochs(ctx.h, ep))
            W.copy_from(A)
            T.rrlu_inplace_device(W, maxrank=r, want_perms=False)
            ctx.synchronize()
            ts = []
            for _ in range(a.reps):
                W.copy_from(A)
                ctx.synchronize()
                t0 = time.perf_counter()
                T.rrlu_inplace_device(W, maxrank=r, want_perms=False)
                ctx.synchronize()
                ts.append(time.perf_counter() - t0)
            ts.sort()
            print(json.dumps({"m": m, "n": n, "r": r, "nb": nb, "epochs": ep,
                              "ms_median": round(ts[len(ts) // 2] * 1e3, 3), "ms_min": round(ts[0] * 1e3, 3)}),
                  flush=True)
        A.free()
        W.free()


if __name__ == "__main__":
    main()
