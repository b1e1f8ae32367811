"""GPU parity: libdcn (HIP kernels on gfx950 + rocBLAS) vs the oracles, through the C-ABI.

Tolerance (north star): fp32 results within |Δ| <= 1e-4 + 1e-4·|ref| of the
reference restatement; M-reductions (∂W, ∂b, ∂W_off, ∂b_off) within
max|Δ|/max|ref| <= 1e-4. Everything here runs on the HIP device (no fallback).
"""
import ctypes

import numpy as np
import pytest

import dcn_oracle as O
import dcn_runtime as rt
import ref_lib as R
from conftest import assert_close, assert_close_reduction, golden_names, load_golden
from deform_conv import DeformConv2dNumpy, dcn_backward_numpy, dcn_forward_numpy

pytestmark = pytest.mark.gpu


def _check(out, off, g, ref_out, ref_off, ref_g, has_bias, what):
    assert_close(out, ref_out, what=f"{what} out")
    assert_close(off, ref_off, what=f"{what} offset")
    assert_close(g["x"], ref_g["x"], what=f"{what} ∂x")
    assert_close(g["offset"], ref_g["offset"], what=f"{what} ∂offset")
    for k in ("weight", "offset_conv.weight", "offset_conv.bias") + (("bias",) if has_bias else ()):
        assert_close_reduction(g[k], ref_g[k], what=f"{what} ∂{k}")


@pytest.mark.parametrize("name", golden_names())
def test_host_api_vs_golden(gpu_handle, name):
    d = load_golden(name)
    out, off = dcn_forward_numpy(d["x"], d["w_off"], d["b_off"], d["w"], d["b"], d["stride"],
                                 d["padding"], handle=gpu_handle)
    g = dcn_backward_numpy(d["x"], off, d["w_off"], d["w"], d["b"] is not None, d["grad_out"],
                           d["stride"], d["padding"], handle=gpu_handle)
    ref_g = {"x": d["f32_grad_x"], "offset": d["f32_grad_offset"], "weight": d["f32_grad_weight"],
             "offset_conv.weight": d["f32_grad_offset_weight"],
             "offset_conv.bias": d["f32_grad_offset_bias"]}
    if d["b"] is not None:
        ref_g["bias"] = d["f32_grad_bias"]
    _check(out, off, g, d["f32_out"], d["f32_off"], ref_g, d["b"] is not None, name)


def _rand_case(seed, B, C, O_, H, W, k=(3, 3), s=(1, 1), p=(1, 1), dil=(1, 1), G=1, off_scale=1.0,
               bias_scale=0.5, bias=True):
    rng = np.random.default_rng(seed)
    N = k[0] * k[1]
    x = rng.standard_normal((B, C, H, W)).astype(np.float32)
    # offsets ~ N(0, off_scale) px (SURVEY §8(d) synthetic inputs)
    wo = (rng.standard_normal((2 * N * G, C, *k)) * off_scale / np.sqrt(C * N)).astype(np.float32)
    bo = rng.uniform(-bias_scale, bias_scale, 2 * N * G).astype(np.float32)
    w = (rng.standard_normal((O_, C, *k)) * np.sqrt(2 / (C * N))).astype(np.float32)
    b = (rng.standard_normal(O_) * 0.1).astype(np.float32) if bias else None
    Ho, Wo = O.out_size(H, W, *k, *s, *p, *dil)
    gout = rng.standard_normal((B, O_, Ho, Wo)).astype(np.float32)
    return dict(x=x, w_off=wo, b_off=bo, w=w, b=b, grad_out=gout, stride=s, padding=p, dil=dil, G=G)


class Dev:
    """Device buffers through the C-ABI memory helpers (no other GPU runtime)."""

    def __init__(self, h):
        self.h, self.ptrs = h, []

    def up(self, a):
        a = np.ascontiguousarray(a, np.float32)
        p = self.h.malloc(a.nbytes)
        self.h.h2d(p, a)
        self.ptrs.append(p)
        return p

    def zeros(self, nbytes):
        p = self.h.malloc(nbytes)
        rt.check(self.h.lib.dcn_memset_zero(self.h.h, ctypes.c_void_p(p), nbytes))
        self.ptrs.append(p)
        return p

    def down(self, p, shape):
        a = np.empty(shape, np.float32)
        self.h.synchronize()
        self.h.d2h(a, p)
        return a

    def free(self):
        for p in self.ptrs:
            self.h.free(p)
        self.ptrs = []


def _device_fwd_bwd(h, c, bwd_flags=None, between=None):
    """dcn_forward + dcn_backward on device buffers, columns reused (DCN_BWD_COL_IN_WS unless
    bwd_flags says otherwise); `between()` runs after the forward, before the backward."""
    if bwd_flags is None:
        bwd_flags = rt.DCN_BWD_COL_IN_WS
    x, wo, bo, w, b, gout = c["x"], c["w_off"], c["b_off"], c["w"], c["b"], c["grad_out"]
    B, C, H, W = x.shape
    O_, _, kh, kw = w.shape
    desc = rt.make_desc(B, C, H, W, O_, (kh, kw), c["stride"], c["padding"], c["dil"], c["G"],
                        bias=b is not None)
    Ho, Wo = rt.out_shape(desc)
    J = wo.shape[0]
    D = Dev(h)
    try:
        px, pwo, pbo, pw = D.up(x), D.up(wo), D.up(bo), D.up(w)
        pb = D.up(b) if b is not None else None
        pout, poff = D.zeros(B * O_ * Ho * Wo * 4), D.zeros(B * J * Ho * Wo * 4)
        wsb = rt.workspace_bytes(desc, True)
        ws = D.zeros(wsb)
        vp = ctypes.c_void_p
        rt.check(h.lib.dcn_forward(h.h, desc, vp(px), vp(pwo), vp(pbo), vp(pw), vp(pb), vp(pout),
                                   vp(poff), vp(ws), wsb), "dcn_forward")
        if between is not None:
            between()
        pgo = D.up(gout)
        pgx, pgw = D.zeros(x.nbytes), D.zeros(w.nbytes)
        pgb = D.zeros(O_ * 4) if b is not None else None
        pgwo, pgbo, pgoff = D.zeros(wo.nbytes), D.zeros(J * 4), D.zeros(B * J * Ho * Wo * 4)
        rt.check(h.lib.dcn_backward(h.h, desc, vp(px), vp(poff), vp(pwo), vp(pw), vp(pgo), vp(pgx),
                                    vp(pgw), vp(pgb), vp(pgwo), vp(pgbo), vp(pgoff), vp(ws), wsb,
                                    bwd_flags), "dcn_backward")
        out, off = D.down(pout, (B, O_, Ho, Wo)), D.down(poff, (B, J, Ho, Wo))
        g = {"x": D.down(pgx, x.shape), "weight": D.down(pgw, w.shape),
             "offset_conv.weight": D.down(pgwo, wo.shape), "offset_conv.bias": D.down(pgbo, (J,)),
             "offset": D.down(pgoff, (B, J, Ho, Wo))}
        if b is not None:
            g["bias"] = D.down(pgb, (O_,))
        return out, off, g
    finally:
        D.free()


def _oracle(c, dev_off=None):
    """Oracle outputs; offsets from the oracle's own conv, everything downstream of them
    conditioned on the device's offsets when given (knife edges, see O.forward)."""
    out, off, cache = O.forward(c["x"], c["w_off"], c["b_off"], c["w"], c["b"], c["stride"],
                                c["padding"], c["dil"], c["G"])
    if dev_off is not None:
        out, _, cache = O.forward(c["x"], c["w_off"], c["b_off"], c["w"], c["b"], c["stride"],
                                  c["padding"], c["dil"], c["G"], offsets=dev_off)
    return out, off, O.backward(cache, c["grad_out"])


@pytest.mark.parametrize("case", [
    dict(seed=1, B=2, C=32, O_=24, H=28, W=28),
    dict(seed=2, B=3, C=16, O_=16, H=20, W=17, s=(2, 2)),
    dict(seed=3, B=1, C=40, O_=8, H=33, W=35, off_scale=3.0, bias_scale=2.0),
    dict(seed=4, B=2, C=8, O_=8, H=64, W=64, s=(2, 2)),           # EDNet conv2 geometry
    dict(seed=5, B=2, C=12, O_=6, H=10, W=12, k=(1, 1), p=(0, 0)),
    dict(seed=6, B=2, C=12, O_=6, H=11, W=12, k=(3, 2), s=(1, 2), p=(1, 0), bias=False),
    dict(seed=7, B=2, C=320, O_=16, H=9, W=10),                     # C > 256: lane-map loop
    dict(seed=8, B=3, C=6, O_=5, H=13, W=11, s=(2, 1)),              # C % 4 != 0: scalar lanes
    # f32-MFMA offset conv fused with the x transpose (3x3 s1 p1, W % 4 == 0, C % 16 == 0)
    dict(seed=9, B=2, C=16, O_=8, H=7, W=4),         # odd H: the last workgroup's 2nd row idle
    dict(seed=10, B=1, C=48, O_=8, H=6, W=60),       # widest row it stages
    dict(seed=11, B=2, C=256, O_=16, H=9, W=56, off_scale=2.0),  # config-3 rows and channels
])
def test_device_api_vs_oracle(gpu_handle, case):
    c = _rand_case(**case)
    out, off, g = _device_fwd_bwd(gpu_handle, c)
    ro, roff, rg = _oracle(c, off)
    _check(out, off, g, ro, roff, rg, c["b"] is not None, str(case))


@pytest.mark.parametrize("dil,G", [((2, 2), 1), ((1, 1), 4), ((2, 2), 4)])
def test_extension_dilation_groups_vs_oracle(gpu_handle, dil, G):
    """Config-5 option set (parity unpinned: checked against our own restatement)."""
    c = _rand_case(21, B=2, C=16, O_=12, H=14, W=14, s=(2, 2), p=(1, 1), dil=dil, G=G)
    out, off, g = _device_fwd_bwd(gpu_handle, c)
    ro, roff, rg = _oracle(c, off)
    _check(out, off, g, ro, roff, rg, True, f"dil={dil} G={G}")


def test_pathological_offsets(gpu_handle):
    """Offsets of tens of pixels: most samples leave the image; bins collect the rest."""
    c = _rand_case(31, B=2, C=8, O_=8, H=40, W=40, off_scale=40.0, bias_scale=30.0)
    out, off, g = _device_fwd_bwd(gpu_handle, c)
    ro, roff, rg = _oracle(c, off)
    _check(out, off, g, ro, roff, rg, True, "huge offsets")


def test_all_samples_out_of_image(gpu_handle):
    """Every sample lands outside the image: out == bias, sampling grads vanish."""
    c = _rand_case(41, B=2, C=4, O_=3, H=12, W=12, off_scale=0.0, bias_scale=0.0)
    c["b_off"][:] = 500.0
    out, off, g = _device_fwd_bwd(gpu_handle, c)
    np.testing.assert_allclose(out, np.broadcast_to(c["b"][None, :, None, None], out.shape))
    assert not np.any(g["offset"]) and not np.any(g["weight"])
    ro, roff, rg = _oracle(c)
    _check(out, off, g, ro, roff, rg, True, "all OOB")


@pytest.mark.parametrize("C,H,W,s,off_scale", [
    (24, 30, 26, (1, 1), 2.0),
    (100, 21, 19, (1, 1), 2.5),   # partial 64-channel LDS slice, ragged 8x8 tiles
    (68, 23, 25, (2, 2), 1.5),    # stride 2: window scale (H-1)/(Wo-1) ~ 2
    (8, 17, 17, (1, 1), 6.0),     # most samples leave the staged window (global path)
    (256, 15, 13, (1, 1), 3.0),   # whole 1-KiB rows (config-3 channel count), ragged tiles
])
def test_channels_last_kernels_match_generic_kernels(gpu_handle, C, H, W, s, off_scale):
    """The channels-last K1/K5 (LDS-staged window + global fallback, lane maps, sample
    bins + gather) and the independent generic kernels (NCHW gathers, global atomics)
    agree: columns bit for bit (same fp32 op order), ∂offset and ∂x to rounding
    (different summation orders)."""
    h = gpu_handle
    c = _rand_case(51, B=3, C=C, O_=4, H=H, W=W, s=s, off_scale=off_scale)
    x, wo, bo = c["x"], c["w_off"], c["b_off"]
    B, C, H, W = x.shape
    desc = rt.make_desc(B, C, H, W, 4, (3, 3), s, (1, 1))
    Ho, Wo = rt.out_shape(desc)
    K, HW = 9 * C, Ho * Wo
    rng = np.random.default_rng(5)
    gcol = rng.standard_normal((B, HW, K)).astype(np.float32)
    vp = ctypes.c_void_p
    res = {}
    for generic in (0, 1):
        D = Dev(h)
        try:
            px, pwo, pbo = D.up(x), D.up(wo), D.up(bo)
            poff = D.zeros(B * 18 * HW * 4)
            rt.check(h.lib.dcn_offset_conv_fwd(h.h, desc, vp(px), vp(pwo), vp(pbo), vp(poff)))
            pcol = D.zeros(B * K * HW * 4)
            rt.check(h.lib.dcn_debug_force_generic(generic))
            rt.check(h.lib.dcn_im2col_fwd(h.h, desc, vp(px), vp(poff), vp(pcol), 0, B))
            pg = D.up(gcol)
            pgx, pgoff = D.zeros(x.nbytes), D.zeros(B * 18 * HW * 4)
            rt.check(h.lib.dcn_col2im_coord_bwd(h.h, desc, vp(px), vp(poff), vp(pg), vp(pgx),
                                                vp(pgoff), 0, B))
            res[generic] = (D.down(pcol, (B, HW, K)), D.down(pgx, x.shape),
                            D.down(pgoff, (B, 18, Ho, Wo)), D.down(poff, (B, 18, Ho, Wo)))
        finally:
            rt.check(h.lib.dcn_debug_force_generic(0))
            D.free()
    col_w, gx_w, goff_w, off_w = res[0]
    col_g, gx_g, goff_g, _ = res[1]
    np.testing.assert_array_equal(col_w, col_g)
    np.testing.assert_allclose(goff_w, goff_g, rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(gx_w, gx_g, rtol=1e-5, atol=1e-5)
    # and both equal the oracle's column block (reference order k = n*C + c per pixel row)
    assert_close(col_w, O.im2col(x, off_w, 3, 3).transpose(0, 2, 1), what="im2col vs oracle")


@pytest.mark.parametrize("B,C,H,W,k,s,p,dil", [
    (2, 64, 20, 20, (3, 3), (1, 1), (1, 1), (1, 1)),   # MFMA kernels
    (3, 100, 21, 19, (3, 3), (1, 1), (1, 1), (1, 1)),  # partial 64-channel group, W % 4 != 0
    (2, 8, 9, 3, (3, 3), (1, 1), (2, 2), (2, 2)),      # dilation 2, rows narrower than a K-step
    (2, 12, 7, 5, (3, 2), (1, 1), (1, 0), (1, 1)),     # rect kernel, Wo < W
    (1, 16, 6, 200, (3, 3), (1, 1), (1, 1), (1, 1)),   # wide rows: 2-row ∂W chunks
    (2, 68, 23, 25, (3, 3), (2, 2), (1, 1), (1, 1)),   # stride 2: VALU kernels only
    (2, 128, 12, 16, (3, 3), (1, 1), (1, 1), (1, 1)),  # ∂W_off on 32x32x2 (C % 128 == 0)
    (3, 256, 9, 12, (3, 3), (1, 1), (1, 1), (1, 1)),   # the same, ragged row chunks
])
def test_offset_conv_bwd_mfma_and_valu_vs_oracle(gpu_handle, B, C, H, W, k, s, p, dil):
    """Offset-conv backward (∂W_off, ∂b_off, ∂x accumulated) on the MFMA kernels (stride 1)
    and on the VALU kernels (dcn_debug_force_generic) against the oracle."""
    h = gpu_handle
    rng = np.random.default_rng(17)
    N = k[0] * k[1]
    x = rng.standard_normal((B, C, H, W)).astype(np.float32)
    wo = (rng.standard_normal((2 * N, C, *k)) / np.sqrt(C * N)).astype(np.float32)
    desc = rt.make_desc(B, C, H, W, 4, k, s, p, dil)
    Ho, Wo = rt.out_shape(desc)
    goff = rng.standard_normal((B, 2 * N, Ho, Wo)).astype(np.float32)
    gx0 = rng.standard_normal(x.shape).astype(np.float32)  # ∂x is accumulated into
    ref_gw, ref_gb, ref_gx = O.offset_conv_backward(x, wo, goff, s, p, dil)
    vp = ctypes.c_void_p
    res = {}
    for generic in (0, 1):
        D = Dev(h)
        try:
            px, pwo, pgoff, pgx = D.up(x), D.up(wo), D.up(goff), D.up(gx0)
            pgw, pgb = D.zeros(wo.nbytes), D.zeros(2 * N * 4)
            rt.check(h.lib.dcn_debug_force_generic(generic))
            rt.check(h.lib.dcn_offset_conv_bwd(h.h, desc, vp(px), vp(pwo), vp(pgoff), vp(pgx),
                                               vp(pgw), vp(pgb)), "dcn_offset_conv_bwd")
            res[generic] = (D.down(pgx, x.shape), D.down(pgw, wo.shape), D.down(pgb, (2 * N,)))
        finally:
            rt.check(h.lib.dcn_debug_force_generic(0))
            D.free()
    for generic, (gx, gw, gb) in res.items():
        tag = f"{'valu' if generic else 'default'}"
        assert_close(gx, gx0 + ref_gx, what=f"{tag} ∂x")
        assert_close_reduction(gw, ref_gw, what=f"{tag} ∂w_off")
        assert_close_reduction(gb, ref_gb, what=f"{tag} ∂b_off")


def test_module_numpy_backend_on_gpu():
    d = load_golden("nonsquare_stride2")
    m = DeformConv2dNumpy(d["x"].shape[1], d["w"].shape[0], 3, 2, 1)
    m.load_state_dict({"weight": d["w"], "bias": d["b"], "offset_conv.weight": d["w_off"],
                       "offset_conv.bias": d["b_off"]})
    out = m(d["x"])
    assert_close(out, d["f32_out"], what="module out")
    gx = m.backward(d["grad_out"])
    assert_close(gx, d["f32_grad_x"], what="module ∂x")
    assert_close_reduction(m.weight.grad, d["f32_grad_weight"], what="module ∂W")
    assert_close_reduction(m.offset_conv.weight.grad, d["f32_grad_offset_weight"],
                           what="module ∂W_off")
    m.eval()
    out2 = m(d["x"])  # no_grad-style forward (train.py:430)
    np.testing.assert_array_equal(out, out2)


def test_empty_batch_host_api(gpu_handle):
    """An empty batch gives empty outputs / ∂x / ∂offset and zero parameter gradients, as
    the reference's ops do, without a launch (the handle is still required)."""
    rng = np.random.default_rng(7)
    x = np.zeros((0, 8, 9, 11), np.float32)
    wo = rng.standard_normal((18, 8, 3, 3)).astype(np.float32)
    bo = np.zeros(18, np.float32)
    w = rng.standard_normal((16, 8, 3, 3)).astype(np.float32)
    b = np.zeros(16, np.float32)
    out, off = dcn_forward_numpy(x, wo, bo, w, b, (2, 2), (1, 1), handle=gpu_handle)
    assert out.shape == (0, 16, 5, 6) and off.shape == (0, 18, 5, 6)
    g = dcn_backward_numpy(x, off, wo, w, True, np.zeros((0, 16, 5, 6), np.float32), (2, 2),
                           (1, 1), handle=gpu_handle)
    assert g["x"].shape == x.shape and g["offset"].shape == off.shape
    for k in ("weight", "bias", "offset_conv.weight", "offset_conv.bias"):
        assert not np.any(g[k]), k


def test_rccl_comm_single_rank_allreduce(gpu_handle):
    """libdcn's RCCL communicator (dcn_comm_* / dcn_allreduce_grads) on a 1-rank world:
    the in-place sum is the identity, on the handle's stream."""
    import dcn_dp
    h = gpu_handle
    uid = dcn_dp.RcclComm.unique_id()
    comm = dcn_dp.RcclComm(h, 1, 0, uid)
    D = Dev(h)
    try:
        g = np.random.default_rng(3).standard_normal(631_570).astype(np.float32)
        p = D.up(g)
        comm.allreduce(p, g.size)
        np.testing.assert_array_equal(D.down(p, g.shape), g)
    finally:
        comm.close()
        D.free()


def test_forward_backward_bitwise_reproducible(gpu_handle):
    """No float atomics on the channels-last path (integer bin counts, fixed-order
    partial sums and shuffle trees): two runs give identical bits."""
    c = _rand_case(71, B=4, C=64, O_=32, H=28, W=28, off_scale=1.5)
    r1 = _device_fwd_bwd(gpu_handle, c)
    r2 = _device_fwd_bwd(gpu_handle, c)
    np.testing.assert_array_equal(r1[0], r2[0])
    np.testing.assert_array_equal(r1[1], r2[1])
    for k in r1[2]:
        np.testing.assert_array_equal(r1[2][k], r2[2][k], err_msg=k)
