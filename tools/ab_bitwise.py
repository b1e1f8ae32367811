"""Bitwise A/B of two libdcn builds on the same seeded inputs (one process per build).

  DCN_LIB=tools/prevlib/libdcn.so python tools/ab_bitwise.py dump gpurun_out/a.npz
  python tools/ab_bitwise.py dump gpurun_out/b.npz
  python tools/ab_bitwise.py cmp gpurun_out/a.npz gpurun_out/b.npz

Cases: config 3 (fp32, full size), config 4 (bf16, one GPU's 64 images) and config 5
(deform_groups 4: the unfused K5 and its sorted sample lists), each forward + backward with
every output kept. Used when a change must leave results bit for bit unchanged (r03: the
bins pipeline rewrite). Test infrastructure; not part of the product."""
import os
import sys

import numpy as np

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [os.path.join(ROOT, "jittor-dcn_amd"), os.path.join(ROOT, "tests"),
                os.path.join(ROOT, "oracle")]


def dump(path):
    import dcn_runtime as rt
    from deform_conv import dcn_backward_numpy, dcn_forward_numpy
    import test_gpu_bf16 as T

    res = {}
    h = rt.Handle(0)
    for tag, (B, C, O_, H, W, s, p, dil, G) in {
            "c3": (64, 256, 256, 56, 56, (1, 1), (1, 1), (1, 1), 1),
            "c5": (64, 512, 512, 14, 14, (2, 2), (1, 1), (2, 2), 4)}.items():
        rng = np.random.default_rng(11)
        J = 18 * G
        x = rng.standard_normal((B, C, H, W)).astype(np.float32)
        wo = (rng.standard_normal((J, C, 3, 3)) / np.sqrt(C * 9)).astype(np.float32)
        bo = rng.uniform(-0.5, 0.5, J).astype(np.float32)
        w = (rng.standard_normal((O_, C, 3, 3)) * np.sqrt(2 / (C * 9))).astype(np.float32)
        b = (rng.standard_normal(O_) * 0.1).astype(np.float32)
        if G == 1 and dil == (1, 1):
            out, off = dcn_forward_numpy(x, wo, bo, w, b, s, p, handle=h)
            gout = rng.standard_normal(out.shape).astype(np.float32)
            g = dcn_backward_numpy(x, off, wo, w, True, gout, s, p, handle=h)
        else:
            out, off, g = _device_f32(h, x, wo, bo, w, b, s, p, dil, G, rng)
        res[f"{tag}_out"], res[f"{tag}_off"] = out, off
        for k, v in g.items():
            res[f"{tag}_g_{k}"] = np.asarray(v)
        print(tag, "done", flush=True)
    bits, _, s = T._case(75, B=64, C=256, O_=256, H=28, W=28)
    out, off, g = T._device(h, bits, s)
    res["c4_out"], res["c4_off"] = out, off
    for k, v in g.items():
        res[f"c4_g_{k}"] = v
    print("c4 done", flush=True)
    h.close()
    np.savez(path, **res)


def _device_f32(h, x, wo, bo, w, b, s, p, dil, G, rng):
    """fp32 forward + backward through the device API (dilation / deform groups)."""
    import ctypes

    import dcn_runtime as rt
    from test_gpu_bf16 import Buf

    B, C, H, W = x.shape
    O_ = w.shape[0]
    J = wo.shape[0]
    desc = rt.make_desc(B, C, H, W, O_, (3, 3), s, p, dil, G)
    Ho, Wo = rt.out_shape(desc)
    gout = rng.standard_normal((B, O_, Ho, Wo)).astype(np.float32)
    D = Buf(h)
    vp = ctypes.c_void_p

    def down(ptr, shape):
        a = np.empty(shape, np.float32)
        h.synchronize()
        rt.check(h.lib.dcn_memcpy_d2h(h.h, a.ctypes.data_as(vp), vp(ptr), a.nbytes))
        return a
    try:
        px, pwo, pbo, pw, pb, pgo = (D.up(a) for a in (x, wo, bo, w, b, gout))
        pout, poff = D.zeros(B * O_ * Ho * Wo * 4), D.zeros(B * J * Ho * Wo * 4)
        wsb = rt.workspace_bytes(desc, True)
        ws = D.zeros(wsb)
        rt.check(h.lib.dcn_forward(h.h, desc, vp(px), vp(pwo), vp(pbo), vp(pw), vp(pb), vp(pout),
                                   vp(poff), vp(ws), wsb))
        gx, gw, gb = D.zeros(x.nbytes), D.zeros(w.nbytes), D.zeros(b.nbytes)
        gwo, gbo, gof = D.zeros(wo.nbytes), D.zeros(bo.nbytes), D.zeros(B * J * Ho * Wo * 4)
        rt.check(h.lib.dcn_backward(h.h, desc, vp(px), vp(poff), vp(pwo), vp(pw), vp(pgo), vp(gx),
                                    vp(gw), vp(gb), vp(gwo), vp(gbo), vp(gof), vp(ws), wsb,
                                    rt.DCN_BWD_COL_IN_WS))
        g = {"x": down(gx, x.shape), "weight": down(gw, w.shape), "bias": down(gb, b.shape),
             "offset_conv.weight": down(gwo, wo.shape), "offset_conv.bias": down(gbo, bo.shape),
             "offset": down(gof, (B, J, Ho, Wo))}
        return down(pout, (B, O_, Ho, Wo)), down(poff, (B, J, Ho, Wo)), g
    finally:
        D.free()


def cmp(a, b):
    A, Bz = np.load(a), np.load(b)
    bad = 0
    for k in sorted(A.files):
        x, y = A[k], Bz[k]
        same = x.shape == y.shape and np.array_equal(x.view(np.uint32), y.view(np.uint32))
        n = 0 if same else int(np.sum(x.view(np.uint32) != y.view(np.uint32)))
        print(f"{k:32s} {'bitwise equal' if same else f'DIFFERS in {n} of {x.size}'}")
        bad += not same
    print("ALL BITWISE EQUAL" if not bad else f"{bad} tensors differ")
    return bad


if __name__ == "__main__":
    if sys.argv[1] == "dump":
        dump(sys.argv[2])
    else:
        sys.exit(1 if cmp(sys.argv[2], sys.argv[3]) else 0)
