"""ctypes binding of oracle/_build/libdcn_ref.so — TEST INFRASTRUCTURE ONLY.

The fp32 C restatement (oracle/dcn_ref.c) of deform_conv.py:56-81 and its
autodiff. Used by tests/ as a second checker, by __graft_entry__.smoke() and by
bench.py's cpu_baseline leg. Never imported by the product package.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "_build", "libdcn_ref.so")


class RefDesc(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int) for n in
                ("B", "C", "H", "W", "O", "kh", "kw", "sh", "sw", "ph", "pw", "dh", "dw", "G",
                 "has_bias")]


_lib = None


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def usable_cpus():
    """Host cores this process may use: the affinity mask, capped by a cgroup CPU quota
    (a shared GPU box reports the whole machine in os.cpu_count())."""
    try:
        n = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        n = os.cpu_count() or 1
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            n = max(1, min(n, -(-int(q) // int(per))))
    except (OSError, ValueError):
        pass
    return n


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        P = ctypes.POINTER(ctypes.c_float)
        D = ctypes.POINTER(RefDesc)
        L.dcnref_forward.argtypes = [D, P, P, P, P, P, P, P]
        L.dcnref_backward.argtypes = [D, P, P, P, P, P, P, P, P, P, P, P]
        L.dcnref_forward_from_offsets.argtypes = [D, P, P, P, P, P]
        L.dcnref_out_shape.argtypes = [D, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)]
        L.dcnref_num_threads.restype = ctypes.c_int
        L.dcnref_set_threads.argtypes = [ctypes.c_int]
        L.dcnref_set_threads(usable_cpus())  # no oversubscription under a CPU quota
        _lib = L
    return _lib


def _p(a):
    if a is None:
        return None
    assert a.dtype == np.float32 and a.flags.c_contiguous
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_float))


def make_desc(x_shape, w_shape, stride, padding, dilation=(1, 1), G=1, has_bias=True):
    B, C, H, W = x_shape
    O, _, kh, kw = w_shape
    return RefDesc(B, C, H, W, O, kh, kw, stride[0], stride[1], padding[0], padding[1],
                   dilation[0], dilation[1], G, int(has_bias))


def out_shape(desc):
    ho, wo = ctypes.c_int(), ctypes.c_int()
    if lib().dcnref_out_shape(ctypes.byref(desc), ctypes.byref(ho), ctypes.byref(wo)):
        raise ValueError("unsupported geometry")
    return ho.value, wo.value


def set_threads(n):
    lib().dcnref_set_threads(int(n))


def num_threads():
    return lib().dcnref_num_threads()


def forward(desc, x, w_off, b_off, w, b):
    Ho, Wo = out_shape(desc)
    J = w_off.shape[0]
    out = np.empty((desc.B, desc.O, Ho, Wo), np.float32)
    off = np.empty((desc.B, J, Ho, Wo), np.float32)
    f = lambda a: None if a is None else np.ascontiguousarray(a, np.float32)
    x, w_off, b_off, w, b = map(f, (x, w_off, b_off, w, b))
    rc = lib().dcnref_forward(ctypes.byref(desc), _p(x), _p(w_off), _p(b_off), _p(w), _p(b),
                              _p(out), _p(off))
    if rc:
        raise RuntimeError(f"dcnref_forward failed ({rc})")
    return out, off


def forward_from_offsets(desc, x, off, w, b):
    """out from GIVEN offsets (deform_conv.py:59-80 without the offset conv)."""
    Ho, Wo = out_shape(desc)
    out = np.empty((desc.B, desc.O, Ho, Wo), np.float32)
    f = lambda a: None if a is None else np.ascontiguousarray(a, np.float32)
    x, off, w, b = map(f, (x, off, w, b))
    rc = lib().dcnref_forward_from_offsets(ctypes.byref(desc), _p(x), _p(off), _p(w), _p(b),
                                           _p(out))
    if rc:
        raise RuntimeError(f"dcnref_forward_from_offsets failed ({rc})")
    return out


def backward(desc, x, off, w_off, w, grad_out):
    f = lambda a: np.ascontiguousarray(a, np.float32)
    x, off, w_off, w, grad_out = map(f, (x, off, w_off, w, grad_out))
    gx = np.empty_like(x)
    gw = np.empty_like(w)
    gb = np.empty(desc.O, np.float32) if desc.has_bias else None
    gwo = np.empty_like(w_off)
    gbo = np.empty(w_off.shape[0], np.float32)
    goff = np.empty_like(off)
    rc = lib().dcnref_backward(ctypes.byref(desc), _p(x), _p(off), _p(w_off), _p(w),
                               _p(grad_out), _p(gx), _p(gw), _p(gb), _p(gwo), _p(gbo), _p(goff))
    if rc:
        raise RuntimeError(f"dcnref_backward failed ({rc})")
    g = {"x": gx, "weight": gw, "offset_conv.weight": gwo, "offset_conv.bias": gbo,
         "offset": goff}
    if gb is not None:
        g["bias"] = gb
    return g
