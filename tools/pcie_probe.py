#!/usr/bin/env python3
"""PCIe / host-copy microbenchmark for the host-pointer API design: pinned vs
pageable DMA rates, hipHostRegister cost, threaded memcpy into touched / untouched memory."""
import ctypes
import json
import threading
import time

import numpy as np

hip = ctypes.CDLL("libamdhip64.so")
hip.hipMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t]
hip.hipHostMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t, ctypes.c_uint]
hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
hip.hipHostRegister.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint]
hip.hipHostUnregister.argtypes = [ctypes.c_void_p]
H2D, D2H = 1, 2
NB = 205_520_896  # config-3 x


def rate(fn, nbytes, reps=3):
    fn()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    return round(nbytes * reps / (time.perf_counter() - t) / 1e9, 2)


res = {}
d = ctypes.c_void_p()
assert hip.hipMalloc(ctypes.byref(d), NB) == 0
pin = ctypes.c_void_p()
assert hip.hipHostMalloc(ctypes.byref(pin), NB, 0) == 0
a = np.ones(NB // 4, np.float32)
res["pinned_h2d_GBs"] = rate(lambda: hip.hipMemcpy(d, pin, NB, H2D), NB)
res["pinned_d2h_GBs"] = rate(lambda: hip.hipMemcpy(pin, d, NB, D2H), NB)
res["pageable_h2d_GBs"] = rate(lambda: hip.hipMemcpy(d, a.ctypes.data, NB, H2D), NB)
res["pageable_d2h_touched_GBs"] = rate(lambda: hip.hipMemcpy(a.ctypes.data, d, NB, D2H), NB)


def fresh_d2h():
    b = np.empty(NB // 4, np.float32)
    hip.hipMemcpy(b.ctypes.data, d, NB, D2H)


res["pageable_d2h_fresh_GBs"] = rate(fresh_d2h, NB)
t = time.perf_counter()
assert hip.hipHostRegister(ctypes.c_void_p(a.ctypes.data), NB, 0) == 0
res["host_register_ms"] = round((time.perf_counter() - t) * 1e3, 2)
res["registered_h2d_GBs"] = rate(lambda: hip.hipMemcpy(d, a.ctypes.data, NB, H2D), NB)
t = time.perf_counter()
hip.hipHostUnregister(ctypes.c_void_p(a.ctypes.data))
res["host_unregister_ms"] = round((time.perf_counter() - t) * 1e3, 2)
pa = np.ctypeslib.as_array((ctypes.c_float * (NB // 4)).from_address(pin.value))
for nt in (1, 4, 8, 16):
    def par(dst_fn):
        dst = dst_fn()
        n = NB // 4
        ths = [threading.Thread(target=np.copyto, args=(dst[i * n // nt:(i + 1) * n // nt],
                                                        a[i * n // nt:(i + 1) * n // nt]))
               for i in range(nt)]
        [t.start() for t in ths]
        [t.join() for t in ths]
    res[f"memcpy_{nt}t_to_pinned_GBs"] = rate(lambda: par(lambda: pa), NB)
    res[f"memcpy_{nt}t_to_fresh_GBs"] = rate(lambda: par(lambda: np.empty(NB // 4, np.float32)), NB)
print(json.dumps(res))
