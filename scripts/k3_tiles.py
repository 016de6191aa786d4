"""K3 (k_dgemm, the blocked Schur update C -= W V) at 8192^2 for nb in (32, 64, 128): device ms by
HIP events (family 22) for the tile shape TCI_DGEMM_TILE selects (0 = by size).
   TCI_DGEMM_TILE=3 python scripts/k3_tiles.py"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tensorcrossinterpolation.jl_amd"))
import tci_amd as T  # noqa: E402
from tci_amd import _lib  # noqa: E402

ctx = _lib.context()
m = n = 8192
Cm = T.DeviceMatrix(m, n, ctx=ctx)
Cm.fill_uniform(seed=3)
out = {"tile": os.environ.get("TCI_DGEMM_TILE", "0")}
for nb in (32, 64, 128):
    W = T.DeviceMatrix(m, nb, ctx=ctx)
    W.fill_uniform(seed=4)
    V = T.DeviceMatrix(nb, n, ctx=ctx)
    V.fill_uniform(seed=5)
    T.schur_update_device(Cm, W, V)
    ctx.set_timing(True)
    for _ in range(10):
        T.schur_update_device(Cm, W, V)
    kms, kn = ctx.kernel_stats(22)
    ctx.set_timing(False)
    ms = kms / kn
    out[f"nb{nb}"] = {"ms": round(ms, 4), "frac_of_spec": round(2.0 * m * n * nb / (ms * 1e-3) / 1e12 / 78.6, 4)}
    W.free()
    V.free()
print(json.dumps(out))
