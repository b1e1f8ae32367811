"""Diagnose libdcn's offset conv forward against the oracle: error pattern per case.
Usage (GPU box): python tools/diag_oc.py"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "jittor-dcn_amd"), os.path.join(ROOT, "oracle")]
import dcn_oracle as O  # noqa: E402
import dcn_runtime as rt  # noqa: E402

h = rt.Handle(0)
vp = ctypes.c_void_p
for (B, C, H, W, s) in [(1, 8, 6, 6, 1), (2, 16, 28, 28, 1), (3, 100, 21, 19, 1), (2, 256, 56, 56, 1)]:
    rng = np.random.default_rng(0)
    x = rng.standard_normal((B, C, H, W)).astype(np.float32)
    wo = (rng.standard_normal((18, C, 3, 3)) / np.sqrt(9 * C)).astype(np.float32)
    bo = rng.standard_normal(18).astype(np.float32)
    desc = rt.make_desc(B, C, H, W, 4, (3, 3), (s, s), (1, 1))
    Ho, Wo = rt.out_shape(desc)
    ref = O.offset_conv(x, wo, bo, (s, s), (1, 1))
    ptrs = []
    def up(a):
        p = h.malloc(a.nbytes); h.h2d(p, np.ascontiguousarray(a)); ptrs.append(p); return p
    px, pwo, pbo = up(x), up(wo), up(bo)
    poff = h.malloc(B * 18 * Ho * Wo * 4); ptrs.append(poff)
    rt.check(h.lib.dcn_offset_conv_fwd(h.h, desc, vp(px), vp(pwo), vp(pbo), vp(poff)))
    off = np.empty((B, 18, Ho, Wo), np.float32)
    h.synchronize(); h.d2h(off, poff)
    for p in ptrs:
        h.free(p)
    err = np.abs(off - ref)
    print(f"B{B} C{C} {H}x{W}: max err {err.max():.3e}; bad per j {(err > 1e-3).sum(axis=(0, 2, 3))}")
    if err.max() > 1e-3:
        bad = err > 1e-3
        print("  bad rows", np.nonzero(bad.any(axis=(0, 1, 3)))[0][:20],
              "bad cols", np.nonzero(bad.any(axis=(0, 1, 2)))[0][:20])
        i = np.unravel_index(np.argmax(err), err.shape)
        print("  worst", i, off[i], ref[i])
        # is it a shifted/permuted version of the right answer?
        for name, cand in [("no bias", ref - bo[None, :, None, None])]:
            print("  vs", name, np.abs(off - cand).max())

# the golden host-API case: offsets and output separately
sys.path.insert(0, os.path.join(ROOT, "tests"))
from conftest import load_golden  # noqa: E402
from deform_conv import dcn_forward_numpy  # noqa: E402
for name in ("config1_28x28", "no_bias"):
    d = load_golden(name)
    out, off = dcn_forward_numpy(d["x"], d["w_off"], d["b_off"], d["w"], d["b"], d["stride"],
                                 d["padding"], handle=h)
    print(name, d["x"].shape, "off err", np.abs(off - d["f32_off"]).max(),
          "out err", np.abs(out - d["f32_out"]).max())
