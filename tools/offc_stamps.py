#!/usr/bin/env python3
"""Phase times of the bf16 offset-conv kernels at config 4 from an OFFC_STAMP=1 diagnostic
build (make alt NAME=ost DEFS=-DOFFC_STAMP=1; run with DCN_LIB=tools/alt/ost/libdcn.so).
Thread 0 of every workgroup stamps s_memrealtime (100 MHz) at its phase boundaries:
  forward (offset_conv_fwd_mfma_bf16_row<4, true>): start, window staged, xT row written,
    k loop done (+ block barrier), partials folded (barrier), end;
  ∂x (offset_dgrad_bf16): start, ∂offset rows staged, k loop done (barrier), end;
  ∂W_off (offset_wgrad_bf16, 2 chunks): start, staged, chunk 0 done, staged, chunks done, end.
Prints per-phase medians and the start-time spread (rounds)."""
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
fn = h.lib.dcn_debug_offc_stamps2
fn.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_int]
KERNELS = [
    ("forward", 64 * 14, ["window staged", "xT row written", "k loop + barrier", "fold barrier",
                          "epilogue"]),
    ("dgrad", 64 * 13, ["goff staged", "k loop + barrier", "epilogue"]),
    ("wgrad", 128 * 2, ["staged 0", "chunk 0 steps", "staged 1", "chunk 1 steps", "partials"]),
]
for which, (name, n, phases) in enumerate(KERNELS):
    buf = (ctypes.c_ulonglong * (n * 8))()
    assert fn(which, ctypes.addressof(buf), n) == 0
    st = np.frombuffer(buf, dtype=np.uint64).reshape(n, 8).astype(np.int64)[:, :len(phases) + 1] * 10
    t0 = st[:, 0].min()
    start = (st[:, 0] - t0) / 1e3
    print(f"== {name}: workgroups {n}; start times us, percentiles 0/25/50/75/100:",
          np.round(np.percentile(start, [0, 25, 50, 75, 100]), 2))
    for i, nm in enumerate(phases):
        d = (st[:, i + 1] - st[:, i]) / 1e3
        print(f"  {nm:18s} median {np.median(d):6.2f} us  p90 {np.percentile(d, 90):6.2f}  max {d.max():6.2f}")
    tot = (st[:, -1] - st[:, 0]) / 1e3
    print(f"  workgroup total    median {np.median(tot):6.2f} us; kernel span {(st[:, -1].max() - t0) / 1e3:.2f} us")
