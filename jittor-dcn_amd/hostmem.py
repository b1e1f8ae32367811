"""Recycled host arrays for the host-pointer path (the NumPy / Jittor-CPU caller).

Every dcn_forward_host / dcn_backward_host call returns new arrays (out, offsets, grads),
as the reference's ops return new Vars. Fresh NumPy memory is not resident yet: the DMA of
a device result into it runs at the page-fault rate, 8.9 GB/s on the MI355X box against
54 GB/s into resident pages (tools/pcie_probe.py). So output arrays come from this pool:
each is a view of a resident block, and the block returns to the pool once nothing
references it any more (a weakref finalizer on the block's owner object, which every view
of the array keeps alive), so the next call of the same shape writes into resident memory.
The arrays behave as ordinary, independent ndarrays to the caller.

With a libdcn handle attached (use_pinned, which the shim does before its first host call)
the blocks are page-locked (dcn_host_alloc): a device-to-host copy into pageable memory runs
as a copy kernel on the CUs through a staging buffer and slows the kernels it overlaps (r03
trace of the pipelined host path: a chunk's offset conv 0.66 ms beside it, ≈0.2 alone);
into page-locked memory it is a DMA. Without a handle (CPU-only use) blocks are plain
resident NumPy memory.
"""
from __future__ import annotations

import ctypes
import threading
import weakref

import numpy as np

_KEEP = 16  # free blocks kept per size (a 4-module stack holds 8+ result blocks of one size)


class _Block:
    """Owner object of one pooled array: numpy takes its memory through the array interface
    (the array's .base), so it lives exactly as long as some view of the memory does."""

    __slots__ = ("__array_interface__", "__weakref__")


class HostPool:
    def __init__(self, keep=_KEEP):
        self.keep = keep
        self._free: dict[int, list[np.ndarray]] = {}
        self._handle = None  # libdcn handle for page-locked blocks (use_pinned)
        # re-entrant: _release runs from a weakref finalizer, which cyclic GC may trigger on
        # this thread while it already holds the lock (inside empty() or _release itself)
        self._lock = threading.RLock()

    def empty(self, shape, dtype=np.float32) -> np.ndarray:
        dtype = np.dtype(dtype)
        shape = tuple(int(s) for s in shape)
        nbytes = int(np.prod(shape, dtype=np.int64)) * dtype.itemsize
        if nbytes < (1 << 20):  # small: no pooling
            return np.empty(shape, dtype)
        with self._lock:
            lst = self._free.get(nbytes)
            store = lst.pop() if lst else None
        if store is None:
            store = self._new_store(nbytes)
        blk = _Block()
        blk.__array_interface__ = {"shape": shape, "typestr": dtype.str,
                                   "data": (store.ctypes.data, False), "version": 3}
        arr = np.asarray(blk)
        weakref.finalize(blk, self._release, nbytes, store)
        return arr

    def use_pinned(self, handle):
        """Allocate later blocks page-locked through libdcn (handle: dcn_runtime.Handle)."""
        with self._lock:
            if self._handle is None or not getattr(self._handle, "h", None):  # none or closed
                self._handle = handle

    def _new_store(self, nbytes):
        h = self._handle
        if h is not None and getattr(h, "h", None):
            p = ctypes.c_void_p()
            if h.lib.dcn_host_alloc(h.h, nbytes, ctypes.byref(p)) == 0 and p.value:
                store = np.ctypeslib.as_array((ctypes.c_uint8 * nbytes).from_address(p.value))
                # the memory goes back to libdcn when the pool drops the block
                f = weakref.finalize(store, h.lib.dcn_host_free, ctypes.c_void_p(p.value))
                f.atexit = False  # at exit the process's pinned pages go with it
                return store
        store = np.empty(nbytes, np.uint8)
        store[::4096] = 0  # make every page resident once
        return store

    def _release(self, nbytes, store):
        with self._lock:
            lst = self._free.setdefault(nbytes, [])
            if len(lst) < self.keep:
                lst.append(store)

    def clear(self):
        with self._lock:
            self._free.clear()


POOL = HostPool()


def use_pinned(handle):
    POOL.use_pinned(handle)


def empty(shape, dtype=np.float32) -> np.ndarray:
    return POOL.empty(shape, dtype)


def empty_like(a) -> np.ndarray:
    return POOL.empty(np.shape(a), np.asarray(a).dtype)
