#!/usr/bin/env python3
"""Phase times of the storing bf16 fused forward (fwd_fused_bf16<true>; `pp`: the ping-pong
fwd_fused_bf16_pp, cycles per segment kind) at config 4, from a
FUSED_STAMP=1 diagnostic build (make alt NAME=st DEFS=-DFUSED_STAMP=1; run with
DCN_LIB=tools/alt/st/libdcn.so). Thread 0 of every workgroup stamps s_memrealtime (100 MHz)
at: start, records done, slice 0..3 windows staged, k loop done, end. Prints, per phase, the
median / 90th percentile / max duration over workgroups, and the spread of start times."""
import ctypes
import os
import sys
here = os.path.dirname(__file__)
sys.path[:0] = [os.path.join(here, "..", d) for d in ("tests", "jittor-dcn_amd", "oracle")]
import numpy as np
import dcn_runtime as rt
import test_gpu_bf16 as T

h = rt.Handle(0)
bits, v, s = T._case(75, B=64, C=256, O_=256, H=28, W=28)
for _ in range(3):
    T._device(h, bits, s)
n = 512
buf = (ctypes.c_ulonglong * (n * 8))()
fn = h.lib.dcn_debug_fused_stamps
fn.argtypes = [ctypes.c_void_p, ctypes.c_int]
assert fn(ctypes.addressof(buf), n) == 0
st = np.frombuffer(buf, dtype=np.uint64).reshape(n, 8).astype(np.int64)
if "pp" in sys.argv[1:]:  # fwd_fused_bf16_pp: per (workgroup, group) shader cycles
    for g in (0, 1):
        s = st[g::2]
        T = s[:, 4].max()
        print(f"group {g}: steps {T}; per step median cycles: gather {np.median(s[:, 0]) / T:.0f} "
              f"multiply {np.median(s[:, 1]) / T:.0f} barriers {np.median(s[:, 2]) / T:.0f}; "
              f"loop {np.median(s[:, 3]):.0f} cycles (max {s[:, 3].max()})")
    sys.exit(0)
t0 = st[:, 0].min()
ns = 10.0  # 100 MHz
names = ["records", "slice0 window", "slice1", "slice2", "slice3 (+ k loop of slice 2)",
         "k loop rest (slice 3)", "epilogue"]
print("start spread us: median %.2f max %.2f" % (np.median(st[:, 0] - t0) * ns / 1e3,
                                               (st[:, 0] - t0).max() * ns / 1e3))
for i, nm in enumerate(names):
    d = (st[:, i + 1] - st[:, i]) * ns / 1e3
    print(f"{nm:32s} median {np.median(d):7.2f} us  p90 {np.percentile(d, 90):7.2f}  max {d.max():7.2f}")
tot = (st[:, 7] - st[:, 0]) * ns / 1e3
print(f"{'workgroup total':32s} median {np.median(tot):7.2f} us  max {tot.max():7.2f}; "
      f"kernel span {(st[:, 7].max() - t0) * ns / 1e3:.2f} us")
