"""Large device -> host copies (tci_abi.cpp d2h_large: 32-MB chunks through two pinned slots, the
host copy threaded) return exactly the bytes of the direct path, at sizes that are not multiples of
the chunk or of the host threads' blocks, into fresh (unfaulted) and reused destinations."""
import ctypes as C

import numpy as np
import pytest

T = pytest.importorskip("tci_amd")
from tci_amd import _lib  # noqa: E402

pytestmark = pytest.mark.gpu


def _ctx():
    return _lib.context()


@pytest.mark.parametrize("m,n", [(9001, 1500), (8192, 4096 + 3)])
def test_large_copy_equals_sliced_direct_copies(m, n):
    ctx = _ctx()
    A = T.DeviceMatrix(m, n, ctx=ctx, ld=m)
    A.fill_uniform(seed=11)
    nbytes = m * n * 8
    assert nbytes >= 64 << 20
    big = np.empty(m * n)  # fresh pages: the copy threads fault them in
    ctx.check(ctx.lib.tci_memcpy_d2h(ctx.h, _lib.ptr(big), A.ptr, nbytes))
    # the same bytes in < 32-MB slices (the direct hipMemcpy path)
    base = A.ptr.value if isinstance(A.ptr, C.c_void_p) else int(A.ptr)
    ref = np.empty(m * n)
    step = (24 << 20) // 8 + 5  # an odd element count per slice
    for o in range(0, m * n, step):
        k = min(step, m * n - o)
        ctx.check(ctx.lib.tci_memcpy_d2h(ctx.h, _lib.ptr(ref[o:o + k]), C.c_void_p(base + 8 * o), 8 * k))
    assert np.array_equal(big.view(np.uint64), ref.view(np.uint64))
    # a reused destination (already faulted in) gets the same bytes again
    A2 = T.DeviceMatrix(m, n, ctx=ctx, ld=m)
    A2.fill_uniform(seed=12)
    ctx.check(ctx.lib.tci_memcpy_d2h(ctx.h, _lib.ptr(big), A2.ptr, nbytes))
    h2 = A2.to_host()
    assert np.array_equal(big.reshape((m, n), order="F").view(np.uint64), np.asarray(h2).view(np.uint64))
    assert not np.array_equal(big.view(np.uint64), ref.view(np.uint64))
    A.free()
    A2.free()
