"""Wall time of one device rrLU per path (small LDS kernel / persistent mid-size grid / pass
pipeline) across sizes: which path wins where.

  python scripts/rrlu_paths.py
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tensorcrossinterpolation.jl_amd"))

import tci_amd as T  # noqa: E402

PATHS = {"small": (1, 1), "mid": (0, 1), "pipeline": (0, 0)}


def main():
    ctx = T.Context(0)
    out = []
    for (m, n, r) in [(120, 120, 12), (128, 128, 64), (256, 256, 64), (512, 512, 64), (1024, 1024, 64),
                      (1024, 1024, 256), (1448, 1448, 128), (2048, 2048, 256), (4096, 4096, 256)]:
        A = T.DeviceMatrix(m, n, ctx=ctx)
        A.fill_uniform(seed=1)
        W = T.DeviceMatrix(m, n, ctx=ctx)
        row = {"m": m, "n": n, "r": r}
        for name, (sm, mid) in PATHS.items():
            ctx.check(ctx.lib.tci_set_rrlu_small(ctx.h, sm))
            ctx.check(ctx.lib.tci_set_rrlu_mid(ctx.h, mid))
            reps = 5
            W.copy_from(A)
            T.rrlu_inplace_device(W, maxrank=r, want_perms=False)
            ctx.synchronize()
            t = 0.0
            for _ in range(reps):
                W.copy_from(A)
                ctx.synchronize()
                t0 = time.perf_counter()
                T.rrlu_inplace_device(W, maxrank=r, want_perms=False)
                t += time.perf_counter() - t0
            row[name + "_ms"] = round(t / reps * 1e3, 3)
        out.append(row)
        print(json.dumps(row), flush=True)
        A.free()
        W.free()


if __name__ == "__main__":
    main()
