"""fp64 MFMA dense kernels alone (bench.py dense_extras): python scripts/dense_bench.py [--k3]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tensorcrossinterpolation.jl_amd"))

import bench  # noqa: E402
import tci_amd as T  # noqa: E402

ctx = T.context(0)
print(json.dumps(bench.dense_extras(T, ctx, only_k3="--k3" in sys.argv)), flush=True)
