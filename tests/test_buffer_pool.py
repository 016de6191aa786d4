"""The recycling of large site-tensor buffers (tensorci2._BufferPool) is unobservable: a replaced
tensor's buffer is reused only when nothing outside the TensorCI2 can still see it."""
import numpy as np

from tci_amd import tensorci2 as T2


def _tensor(pool, n=(3 << 20)):
    buf = pool.take(n)  # 24 MB: above the recycling threshold
    buf[:] = 1.0
    return buf[:n].reshape((1024, 3, n // 3072), order="F")


def test_unobserved_buffer_is_recycled():
    pool = T2._BufferPool()
    holder = [_tensor(pool)]
    pool.give_back(holder)
    assert holder == [None]
    assert sum(len(v) for v in pool.free.values()) == 1
    again = pool.take(3 << 20)
    assert sum(len(v) for v in pool.free.values()) == 0
    assert again.size == 3 << 20


def test_held_view_blocks_recycling():
    pool = T2._BufferPool()
    t = _tensor(pool)
    mine = t[:, 0, :]  # the user keeps a view of the tensor
    pool.give_back([t])
    del t
    assert sum(len(v) for v in pool.free.values()) == 0
    assert float(mine[0, 0]) == 1.0


def test_held_tensor_blocks_recycling():
    pool = T2._BufferPool()
    t = _tensor(pool)
    kept = t
    pool.give_back([t])
    del t
    assert sum(len(v) for v in pool.free.values()) == 0
    fresh = pool.take(3 << 20)
    fresh[:] = 2.0
    assert float(kept[0, 0, 0]) == 1.0  # never handed out again while held


def test_foreign_and_small_arrays_are_ignored():
    pool = T2._BufferPool()
    pool.give_back([np.zeros(4 << 20), np.zeros(10), None])
    assert pool.free == {} and pool.bytes == 0


def test_cap_bounds_the_pool():
    pool = T2._BufferPool()
    pool._CAP = 30 << 20
    a, b = [_tensor(pool)], [_tensor(pool)]
    pool.give_back(a)
    pool.give_back(b)
    assert sum(len(v) for v in pool.free.values()) == 1 and pool.bytes <= pool._CAP
