"""Timing of the ComplexF64 rrLU (tci_rrlu_c128_h) at (m, n, r): wall time of the call minus the
host->device upload (measured separately), algorithmic GFLOP/s (8 flops per complex
multiply-subtract) and bytes (32 B per trailing element per pivot). Run under rocprofv3
--kernel-trace --stats for the per-kernel split."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tensorcrossinterpolation.jl_amd"))

import numpy as np  # noqa: E402

import tci_amd as T  # noqa: E402


def main():
    sizes = [(4096, 4096, 256), (8192, 8192, 256)]
    if len(sys.argv) > 1:
        sizes = [tuple(int(v) for v in a.split(",")) for a in sys.argv[1:]]
    ctx = T.Context(0)
    for m, n, r in sizes:
        rng = np.random.default_rng(0)
        A = np.asfortranarray(rng.random((m, n)) + 1j * rng.random((m, n)))
        T.rrlu(A[:64, :64], ctx=ctx)  # warm-up
        ts = []
        for _ in range(3):
            t0 = time.perf_counter()
            lu = T.rrlu(A, maxrank=r, reltol=0.0, ctx=ctx)
            ts.append(time.perf_counter() - t0)
        t0 = time.perf_counter()
        T.rrlu(A, maxrank=0, ctx=ctx)  # upload + init only
        tup = time.perf_counter() - t0
        k = np.arange(1, lu.npivot + 1, dtype=np.float64)
        el = ((m - k) * (n - k)).sum()
        t = min(ts) - tup
        print(f"complex rrLU {m}x{n} r={lu.npivot}: {t * 1e3:.1f} ms (call {min(ts) * 1e3:.1f}, "
              f"upload {tup * 1e3:.1f}); {8 * el / t / 1e9:.0f} GFLOP/s, {32 * el / t / 1e9:.0f} GB/s",
              flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
