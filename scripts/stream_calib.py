"""Stream read/copy bandwidth vs grid size on one MI355X (roofline calibration)."""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tensorcrossinterpolation.jl_amd"))
import tci_amd as T

ctx = T.context(0)
for mb in (512, 2048):
    n = mb * 1024 * 1024 // 8
    a = T.DeviceMatrix(n, 1, ctx=ctx)
    b = T.DeviceMatrix(n, 1, ctx=ctx)
    a.fill_uniform(1)
    for grid in (512, 1024, 2048, 4096, 8192, 16384, 65536, 262144):
        r, cp = C.c_double(), C.c_double()
        ctx.check(ctx.lib.tci_diag_stream_d(ctx.h, a.ptr, b.ptr, n, 10, grid, C.byref(r), C.byref(cp)))
        print(f"{mb} MiB grid {grid:7d}: read {8 * n / r.value / 1e6:7.1f} GB/s  copy {16 * n / cp.value / 1e6:7.1f} GB/s", flush=True)
    a.free()
    b.free()
