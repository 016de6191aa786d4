"""One small rrLU and exit, to bisect exit-time faults under rocprofv3 (TCI_RRLU_MID / _SMALL pick
the path). python scripts/exit_probe.py [m]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "tensorcrossinterpolation.jl_amd"))
import tci_amd as T  # noqa: E402

m = int(sys.argv[1]) if len(sys.argv) > 1 else 600
A = np.random.default_rng(0).random((m, m))
lu = T.rrlu(A)
print("rank", lu.npivots() if callable(getattr(lu, "npivots", None)) else lu, flush=True)
