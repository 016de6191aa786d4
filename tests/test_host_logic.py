"""CPU-only tests of the host side: index-set algebra, convergence logic, and that the C-ABI
library loads and exports every symbol declared in include/tci_hip.h (no compute calls)."""
import ctypes
import os
import re

import numpy as np
import pytest

import oracle_lib as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_header_symbols_exported():
    from tci_amd import _lib
    if not os.path.exists(_lib.LIB_PATH):
        import subprocess
        subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "tensorcrossinterpolation.jl_amd", "csrc")])
    with open(os.path.join(ROOT, "include", "tci_hip.h")) as fh:
        hdr = fh.read()
    names = sorted(set(re.findall(r"^\w[\w\s\*]*?\b(tci_\w+)\s*\(", hdr, flags=re.M)))
    assert len(names) >= 20, names
    lib = ctypes.CDLL(_lib.LIB_PATH)
    for n in names:
        assert hasattr(lib, n), n
    assert set(_lib.SIGNATURES) <= set(names)


def test_product_never_imports_oracle():
    pkg = os.path.join(ROOT, "tensorcrossinterpolation.jl_amd")
    for dp, _, fns in os.walk(pkg):
        for fn in fns:
            if fn.endswith((".py", ".cpp", ".hip", ".h", ".jl")):
                with open(os.path.join(dp, fn), errors="replace") as fh:
                    txt = fh.read()
                assert "oracle_lib" not in txt and "liboracle" not in txt, fn


def test_kronecker_orders():
    from tci_amd import kronecker_left, kronecker_right
    I = np.array([[1, 2], [3, 4], [5, 6]], np.int32)
    k = kronecker_right(I, 3)
    # Iset fastest (tensorci2.jl:516)
    assert k.tolist()[:4] == [[1, 2, 1], [3, 4, 1], [5, 6, 1], [1, 2, 2]]
    k2 = kronecker_left(3, I)
    assert k2.tolist()[:4] == [[1, 1, 2], [2, 1, 2], [3, 1, 2], [1, 3, 4]]
    multiset = np.array([[1, 2, 3, 4, 5]] * 5, np.int32)
    for ci in kronecker_right(multiset, 4):  # test_tensorci2.jl:9-25
        assert list(ci[:5]) == [1, 2, 3, 4, 5] and 1 <= ci[5] <= 4
    for di in kronecker_left(4, multiset):
        assert 1 <= di[0] <= 4 and list(di[1:]) == [1, 2, 3, 4, 5]


def test_union_first_seen_order():
    from tci_amd import union_sets
    a = np.array([[3, 1], [1, 1], [3, 1], [2, 2]], np.int32)
    b = np.array([[2, 2], [0, 9], [1, 1], [7, 7]], np.int32)
    assert union_sets(a, b).tolist() == [[3, 1], [1, 1], [2, 2], [0, 9], [7, 7]]
    assert union_sets(a, None).tolist() == [[3, 1], [1, 1], [2, 2]]


def test_convergencecriterion_truth_table(kats):
    from tci_amd import convergencecriterion
    for c in kats["convergencecriterion"]["cases"]:
        assert convergencecriterion(c["ranks"], c["errors"], c["ngp"], c["tol"], c["maxbonddim"],
                                    c["ncheck"]) == c["expect"]


def test_forwardsweep():
    from tci_amd import forwardsweep
    assert forwardsweep("forward", 2) and forwardsweep("backandforth", 1)
    assert not forwardsweep("backandforth", 2)


def test_jl_max_semantics():
    from tci_amd.tensorci2 import jl_max
    assert np.isnan(jl_max(1.0, np.nan)) and np.isnan(jl_max(np.nan, 1.0))
    assert jl_max(-0.0, 0.0) == 0.0 and not np.signbit(jl_max(-0.0, 0.0))
    assert jl_max(2.0, 3.0) == 3.0


def test_oracle_generator_matches_spec():
    # splitmix64 stream shared with the device fill (tci_fill_uniform_d)
    a = O.fill_uniform(4, seed=0)
    assert np.all((a >= 0) & (a < 1)) and len(set(a.tolist())) == 4


def test_no_gpu_raises_loudly():
    import tci_amd
    try:
        import torch
        has = torch.cuda.is_available()
    except Exception:
        has = False
    if has:
        pytest.skip("GPU present")
    with pytest.raises(tci_amd.TCIError):
        tci_amd.Context(0)


@pytest.mark.parametrize("mode", ["pointwise", "threads", "vectorized", "batch"])
@pytest.mark.parametrize("M", [0, 1])
def test_host_function_batch_layout_vs_oracle(mode, M):
    """HostFunctionEvaluator's host batch (the array its callback hands the library) has the
    layout of _batchevaluate_dispatch (batcheval.jl:154-174): element (i, c, j) at i + m c + m D j,
    bitwise the oracle's batch evaluation of the same integer-exact f (f = sum(x), kind 0)."""
    from tci_amd.hostfunction import HostFunctionEvaluator
    ld = [3, 4, 5, 2, 3]
    ev = object.__new__(HostFunctionEvaluator)  # host side only: no device context
    ev.localdims, ev.L, ev._pool = ld, len(ld), None
    ev.threads, ev.vectorized, ev.is_batch = (4 if mode == "threads" else 1), mode == "vectorized", mode == "batch"
    if mode == "vectorized":
        ev.f = lambda X: X.sum(axis=1).astype(float)
    elif mode == "batch":
        def fb(I, J, MM):
            s = I.sum(1)[:, None] + J.sum(1)[None, :]
            if MM == 0:
                return s.astype(float)
            d = ld[I.shape[1]]
            return (s[:, None, :] + np.arange(1, d + 1)[None, :, None]).astype(float)
        ev.f = fb
    else:
        ev.f = lambda x: float(sum(x))
    rng = np.random.default_rng(M)
    nl = 2
    I = np.stack([rng.integers(1, d + 1, 23) for d in ld[:nl]], 1).astype(np.int32)
    J = np.stack([rng.integers(1, d + 1, 17) for d in ld[nl + M:]], 1).astype(np.int32)
    got = ev._batch_host(I, J, M)
    ref, mx = O.batcheval(0, [0.0], ld, I, J, M)
    D = ld[nl] if M else 1
    assert np.array_equal(got, ref.reshape((23 * D, 17), order="F"))
    out, gmx = ev.pi(I, J, M)
    assert gmx == mx
    if ev._pool is not None:
        ev._pool.shutdown()


def test_contraction_f_complex_into_real_raises():
    """a Float64 Contraction whose f returns a complex value with a nonzero imaginary part
    throws InexactError in the reference (`res .= obj.f.(res)` into a Float64 array,
    contraction.jl:571); real-valued complex results and real f pass through."""
    from tci_amd.contraction import InexactError, _elementwise
    vals = np.linspace(0.1, 1.0, 6).reshape(2, 3)
    with pytest.raises(InexactError):
        _elementwise(lambda x: np.exp(1j * x), vals)
    with pytest.raises(InexactError):  # the element-by-element path (f not vectorised)
        _elementwise(lambda x: complex(x, 1.0) if isinstance(x, float) else None, vals)
    assert np.array_equal(_elementwise(lambda x: x + 0j, vals), vals)
    assert np.array_equal(_elementwise(lambda x: 2 * x, vals), 2 * vals)
    c = _elementwise(lambda x: np.exp(1j * x), vals, np.complex128)
    assert np.allclose(c, np.exp(1j * vals))
