"""Repeatability of batch evaluation (CP kind, MFMA GEMM): the same (I, J) evaluated repeatedly,
interleaved with other sizes, must give bitwise the same Pi and max|Pi|."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tensorcrossinterpolation.jl_amd"))

import numpy as np  # noqa: E402

import tci_amd as T  # noqa: E402

rng = np.random.default_rng(2)
K, L, d = 256, 12, 32
f = T.cp_function(0.5 + rng.random((K, L, d)))
bad = 0
for (m, n, nl) in [(32, 32, 1), (1024, 32, 2), (1024, 1024, 6), (8192, 256, 3), (300, 5000, 5), (96, 96, 6)]:
    I = rng.integers(1, d + 1, size=(m, nl)).astype(np.int32)
    J = rng.integers(1, d + 1, size=(n, L - nl)).astype(np.int32)
    ref, mref = f.pi(I, J, 0)
    ref = ref.copy()
    for rep in range(4):
        # an unrelated evaluation in between
        f.pi(rng.integers(1, d + 1, size=(rep * 100 + 7, nl)).astype(np.int32), J[:50], 0)
        got, mg = f.pi(I, J, 0)
        if not (np.array_equal(got, ref) and mg == mref):
            bad += 1
            diff = np.argwhere(got != ref)
            print(f"m={m} n={n} nl={nl} rep={rep}: {len(diff)} entries differ, first {diff[:3].tolist()}, "
                  f"max {mg} vs {mref}", flush=True)
print("pi repeat: differing evaluations", bad)
