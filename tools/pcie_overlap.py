#!/usr/bin/env python3
"""Can the host path's transfers overlap each other and the kernels?

Times, for a config-3-sized tensor (205 MB), pageable and pinned hipMemcpyAsync:
  * host time of the async call itself (does a pageable copy block the caller?);
  * H2D and D2H issued together on two streams, from one thread and from two threads;
  * H2D beside a ~10 ms GEMM running on another stream.
Prints one JSON object. Test infrastructure only."""
import ctypes
import json
import threading
import time

import numpy as np
import torch

hip = ctypes.CDLL("libamdhip64.so")
vp, sz = ctypes.c_void_p, ctypes.c_size_t
hip.hipMalloc.argtypes = [ctypes.POINTER(vp), sz]
hip.hipHostMalloc.argtypes = [ctypes.POINTER(vp), sz, ctypes.c_uint]
hip.hipMemcpyAsync.argtypes = [vp, vp, sz, ctypes.c_int, vp]
hip.hipStreamCreate.argtypes = [ctypes.POINTER(vp)]
hip.hipStreamSynchronize.argtypes = [vp]
H2D, D2H = 1, 2
NB = 205_520_896


def mk_stream():
    s = vp()
    assert hip.hipStreamCreate(ctypes.byref(s)) == 0
    return s


def dev(n):
    p = vp()
    assert hip.hipMalloc(ctypes.byref(p), n) == 0
    return p


def pinned(n):
    p = vp()
    assert hip.hipHostMalloc(ctypes.byref(p), n, 0) == 0
    return p


s1, s2 = mk_stream(), mk_stream()
d_in, d_out = dev(NB), dev(NB)
pg_in = np.ones(NB // 4, np.float32)
pg_out = np.ones(NB // 4, np.float32)
pn_in, pn_out = pinned(NB), pinned(NB)
ctypes.memset(pn_in, 1, NB)
ctypes.memset(pn_out, 1, NB)


def best(fn, reps=4):
    fn()
    out = []
    for _ in range(reps):
        t = time.perf_counter()
        r = fn()
        out.append((time.perf_counter() - t, r))
    return min(out, key=lambda v: v[0])


res = {}
for kind, src, dst in (("pageable", pg_in.ctypes.data, pg_out.ctypes.data),
                       ("pinned", pn_in.value, pn_out.value)):
    def h2d(s=s1):
        t = time.perf_counter()
        hip.hipMemcpyAsync(d_in, src, NB, H2D, s)
        call = time.perf_counter() - t
        hip.hipStreamSynchronize(s)
        return call

    def d2h(s=s2):
        t = time.perf_counter()
        hip.hipMemcpyAsync(dst, d_out, NB, D2H, s)
        call = time.perf_counter() - t
        hip.hipStreamSynchronize(s)
        return call

    def both_one_thread():
        hip.hipMemcpyAsync(d_in, src, NB, H2D, s1)
        hip.hipMemcpyAsync(dst, d_out, NB, D2H, s2)
        hip.hipStreamSynchronize(s1)
        hip.hipStreamSynchronize(s2)

    def both_two_threads():
        ts = [threading.Thread(target=h2d), threading.Thread(target=d2h)]
        [t.start() for t in ts]
        [t.join() for t in ts]

    t, call = best(h2d)
    res[f"{kind}_h2d_ms"], res[f"{kind}_h2d_call_ms"] = round(t * 1e3, 2), round(call * 1e3, 2)
    t, call = best(d2h)
    res[f"{kind}_d2h_ms"], res[f"{kind}_d2h_call_ms"] = round(t * 1e3, 2), round(call * 1e3, 2)
    res[f"{kind}_both_1thread_ms"] = round(best(both_one_thread)[0] * 1e3, 2)
    res[f"{kind}_both_2threads_ms"] = round(best(both_two_threads)[0] * 1e3, 2)

    # beside a GEMM on a torch stream
    a = torch.randn(6144, 6144, device="cuda")
    ts = torch.cuda.Stream()

    def gemm():
        with torch.cuda.stream(ts):
            for _ in range(2):
                a @ a
        ts.synchronize()

    res["gemm_alone_ms"] = round(best(gemm)[0] * 1e3, 2)

    def gemm_and_h2d():
        with torch.cuda.stream(ts):
            for _ in range(2):
                a @ a
        hip.hipMemcpyAsync(d_in, src, NB, H2D, s1)
        hip.hipMemcpyAsync(dst, d_out, NB, D2H, s2)
        hip.hipStreamSynchronize(s1)
        hip.hipStreamSynchronize(s2)
        ts.synchronize()

    res[f"{kind}_gemm_plus_both_ms"] = round(best(gemm_and_h2d)[0] * 1e3, 2)
print(json.dumps(res))
