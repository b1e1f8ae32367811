"""CPU: the recycled host-array pool of the host-pointer path (jittor-dcn_amd/hostmem.py).
Arrays it hands out must behave as independent ndarrays: no two live arrays share memory, a
view keeps its block out of the pool, and a block is reused only once nothing refers to it."""
import gc

import numpy as np

import hostmem


def test_pool_recycles_only_dead_blocks():
    pool = hostmem.HostPool(keep=2)
    shape = (4, 256, 512)  # 2 MiB: pooled
    a = pool.empty(shape)
    a[...] = 1.0
    pa = a.ctypes.data
    b = pool.empty(shape)  # a is alive: a new block
    assert b.ctypes.data != pa
    v = a[1:3]  # a view keeps a's block alive
    del a
    gc.collect()
    c = pool.empty(shape)
    assert c.ctypes.data not in (pa, b.ctypes.data)
    np.testing.assert_array_equal(v, 1.0)  # untouched by later allocations
    del v
    gc.collect()
    d = pool.empty(shape)  # now a's block is free again
    assert d.ctypes.data == pa
    assert d.shape == shape and d.dtype == np.float32 and d.flags.c_contiguous
    assert d.flags.writeable


def test_pool_small_and_other_dtypes():
    pool = hostmem.HostPool()
    s = pool.empty((3, 5))  # small: plain np.empty
    assert s.shape == (3, 5) and s.base is None
    x = pool.empty((1 << 19,), np.float64)  # 4 MiB float64
    assert x.dtype == np.float64 and x.nbytes == 1 << 22
    y = hostmem.empty_like(x)
    assert y.dtype == np.float64 and y.shape == x.shape and y.ctypes.data != x.ctypes.data
