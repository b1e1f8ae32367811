"""DCN_BF16 (BASELINE config 4's dtype): bf16 tensors at the C-ABI, bf16 columns / GEMM
operands inside, fp32 coordinates, accumulation and reductions.

Oracle: the fp32/f64 restatement run on the bf16-rounded inputs, its sampling conditioned
on the device's own bf16 offsets (knife edges, see test_gpu_parity). Tolerance (SURVEY
§8(d): 1e-4 is unattainable in bf16, ≈1e-2 relative): elementwise, every element of every
tensor within BF16_ATOL·rms(ref) + BF16_RTOL·|ref| (assert_bf16_close)."""
from __future__ import annotations

import ctypes

import numpy as np
import pytest

import dcn_oracle as O
import dcn_runtime as rt
import ref_lib as R

pytestmark = pytest.mark.gpu
BF16_TOL = 1e-2  # measured r01: 2-4e-3 (about one bf16 ulp) on every tensor
# Elementwise bf16 bound: |Δ| <= BF16_ATOL·rms(ref) + BF16_RTOL·|ref|
# for EVERY element, so a localised wrong element (a corrupted column row, a wrong pixel)
# fails even when the tensor's max-norm error stays small. rtol = 4 bf16 ulps (2^-6): the
# device rounds its inputs' products, columns and result to bf16 (a half ulp, 2^-9, each);
# atol scales with the tensor's RMS because the column roundings accumulate over K-long
# sums whose result can cancel to near zero (an absolute, not relative, error there).
BF16_RTOL = 2.0 ** -6
BF16_ATOL = 2.0 ** -5


def to_bf16(a):
    """float32 -> bf16 bits (round to nearest even; inputs here are finite)."""
    u = np.ascontiguousarray(a, np.float32).view(np.uint32).astype(np.uint64)
    return ((u + 0x7FFF + ((u >> 16) & 1)) >> 16).astype(np.uint16)


def from_bf16(b):
    return (np.asarray(b, np.uint16).astype(np.uint32) << 16).view(np.float32)


def assert_bf16_close(a, ref, what):
    """Elementwise: |Δ| <= BF16_ATOL·rms(ref) + BF16_RTOL·|ref| (see BF16_RTOL)."""
    a = np.asarray(a, np.float64)
    r = np.asarray(ref, np.float64)
    assert a.shape == r.shape, f"{what}: shape {a.shape} vs {r.shape}"
    rms = float(np.sqrt(np.mean(r * r))) if r.size else 0.0
    lim = BF16_ATOL * max(rms, 1e-30) + BF16_RTOL * np.abs(r)
    d = np.abs(a - r)
    bad = ~(d <= lim)
    if bad.any():
        i = np.unravel_index(np.argmax(d / lim), a.shape)
        raise AssertionError(f"{what}: {int(bad.sum())} / {a.size} elements past the bf16 bound; "
                             f"worst at {i}: got {a[i]!r} want {r[i]!r} (|Δ|/bound "
                             f"{float(d[i] / lim[i]):.2f}, rms {rms:.3e})")
    return float(np.max(d / lim)) if a.size else 0.0


def rel_err(a, ref):
    ref = np.asarray(ref, np.float64)
    return float(np.max(np.abs(np.asarray(a, np.float64) - ref)) / max(np.max(np.abs(ref)), 1e-30))


class Buf:
    def __init__(self, h):
        self.h, self.ptrs = h, []

    def up(self, bits):
        bits = np.ascontiguousarray(bits)
        p = self.h.malloc(bits.nbytes)
        rt.check(self.h.lib.dcn_memcpy_h2d(self.h.h, ctypes.c_void_p(p),
                                           bits.ctypes.data_as(ctypes.c_void_p), bits.nbytes))
        self.ptrs.append(p)
        return p

    def zeros(self, nbytes):
        p = self.h.malloc(nbytes)
        rt.check(self.h.lib.dcn_memset_zero(self.h.h, ctypes.c_void_p(p), nbytes))
        self.ptrs.append(p)
        return p

    def down(self, p, shape):
        a = np.empty(shape, np.uint16)
        self.h.synchronize()
        rt.check(self.h.lib.dcn_memcpy_d2h(self.h.h, a.ctypes.data_as(ctypes.c_void_p),
                                           ctypes.c_void_p(p), a.nbytes))
        return from_bf16(a)

    def free(self):
        for p in self.ptrs:
            self.h.free(p)


def _case(seed, B, C, O_, H, W, s=(1, 1), off_scale=1.0, k=(3, 3), p=(1, 1)):
    rng = np.random.default_rng(seed)
    N = k[0] * k[1]
    x = rng.standard_normal((B, C, H, W)).astype(np.float32)
    wo = (rng.standard_normal((2 * N, C, *k)) * off_scale / np.sqrt(C * N)).astype(np.float32)
    bo = rng.uniform(-0.5, 0.5, 2 * N).astype(np.float32)
    w = (rng.standard_normal((O_, C, *k)) * np.sqrt(2 / (C * N))).astype(np.float32)
    b = (rng.standard_normal(O_) * 0.1).astype(np.float32)
    Ho, Wo = O.out_size(H, W, *k, *s, *p)
    gout = rng.standard_normal((B, O_, Ho, Wo)).astype(np.float32)
    c = dict(x=x, w_off=wo, b_off=bo, w=w, b=b, grad_out=gout)
    bits = {k_: to_bf16(v) for k_, v in c.items()}
    vals = {k_: from_bf16(v) for k_, v in bits.items()}  # what the device actually sees
    return bits, vals, s


def _device(h, bits, s, pad=(1, 1), comm=None):
    B, C, H, W = bits["x"].shape
    O_, _, kh, kw = bits["w"].shape
    J = bits["w_off"].shape[0]
    desc = rt.make_desc(B, C, H, W, O_, (kh, kw), s, pad, dtype=rt.DCN_BF16)
    Ho, Wo = rt.out_shape(desc)
    D = Buf(h)
    vp = ctypes.c_void_p
    try:
        p = {k: D.up(v) for k, v in bits.items()}
        pout, poff = D.zeros(B * O_ * Ho * Wo * 2), D.zeros(B * J * Ho * Wo * 2)
        wsb = rt.workspace_bytes(desc, True)
        ws = D.zeros(wsb)
        rt.check(h.lib.dcn_forward(h.h, desc, vp(p["x"]), vp(p["w_off"]), vp(p["b_off"]),
                                   vp(p["w"]), vp(p["b"]), vp(pout), vp(poff), vp(ws), wsb))
        g = {k: D.zeros(v.nbytes) for k, v in bits.items() if k != "grad_out"}
        pgoff = D.zeros(B * J * Ho * Wo * 2)
        if comm is not None:
            h.set_comm(comm)
        rt.check(h.lib.dcn_backward(h.h, desc, vp(p["x"]), vp(poff), vp(p["w_off"]), vp(p["w"]),
                                    vp(p["grad_out"]), vp(g["x"]), vp(g["w"]), vp(g["b"]),
                                    vp(g["w_off"]), vp(g["b_off"]), vp(pgoff), vp(ws), wsb,
                                    rt.DCN_BWD_COL_IN_WS))
        out = D.down(pout, (B, O_, Ho, Wo))
        off = D.down(poff, (B, J, Ho, Wo))
        grads = {"x": D.down(g["x"], bits["x"].shape), "weight": D.down(g["w"], bits["w"].shape),
                 "bias": D.down(g["b"], bits["b"].shape),
                 "offset_conv.weight": D.down(g["w_off"], bits["w_off"].shape),
                 "offset_conv.bias": D.down(g["b_off"], bits["b_off"].shape),
                 "offset": D.down(pgoff, (B, J, Ho, Wo))}
        return out, off, grads
    finally:
        if comm is not None:
            h.set_comm(None)
        D.free()


def _bf16_sweep(i):
    """Seeded random bf16 geometries (3x3, pad 1, stride 1-2): every channel instantiation."""
    rng = np.random.default_rng(500 + i)
    C = (4, 20, 48, 96, 160, 256)[i]
    return dict(seed=600 + i, B=int(rng.integers(1, 4)), C=C, O_=int(rng.choice([8, 64, 256])),
                H=int(rng.integers(6, 22)), W=int(rng.integers(6, 22)),
                s=(int(rng.integers(1, 3)), int(rng.integers(1, 3))),
                off_scale=float(rng.choice([1.0, 2.5])))


@pytest.mark.parametrize("case", [
    dict(seed=1, B=2, C=64, O_=32, H=20, W=20),
    dict(seed=2, B=3, C=32, O_=16, H=17, W=15, s=(2, 2)),
    dict(seed=3, B=1, C=256, O_=64, H=14, W=14, off_scale=2.0),
    dict(seed=4, B=2, C=12, O_=8, H=11, W=13),
    # the bf16 MFMA offset-conv backward (C % 64, H·W % 8, W % 4): ragged 5-row ∂W_off
    # chunks (60 px: a 4-pixel tail), W = 4 (a k-step spans four rows), 3 channel waves
    dict(seed=5, B=3, C=64, O_=32, H=10, W=12, off_scale=2.0),
    dict(seed=6, B=2, C=128, O_=64, H=8, W=4),
    dict(seed=7, B=1, C=192, O_=16, H=13, W=16, off_scale=2.5),
    # C = O = 256: the ∂columns on dcol_bf16 (K % 256 == 0, O == 256): 507 pixels (a
    # 59-pixel last chunk), and stride 2 with 144 pixels (a 16-pixel last chunk)
    dict(seed=8, B=3, C=256, O_=256, H=13, W=13),
    dict(seed=9, B=2, C=256, O_=256, H=17, W=15, s=(2, 2), off_scale=2.0),
] + [_bf16_sweep(i) for i in range(6)])
def test_bf16_forward_backward_vs_oracle(gpu_handle, case):
    bits, v, s = _case(**case)
    out, off, g = _device(gpu_handle, bits, s)
    _, roff, _ = O.forward(v["x"], v["w_off"], v["b_off"], v["w"], v["b"], s, (1, 1))
    assert rel_err(off, roff) <= BF16_TOL, "offsets"
    # the offset conv's products are exact (bf16 inputs) and summed in fp32, so the only
    # visible error is the final rounding of the offsets to bf16 (half an ulp, 2^-9)
    assert np.all(np.abs(off - roff) <= 2.0 ** -8 * np.abs(roff) + 1e-6), "offsets past 1 ulp"
    ro, _, cache = O.forward(v["x"], v["w_off"], v["b_off"], v["w"], v["b"], s, (1, 1),
                             offsets=off)  # condition on the device's bf16 offsets
    rg = O.backward(cache, v["grad_out"])
    assert_bf16_close(out, ro, "out")
    for k in ("x", "weight", "bias", "offset_conv.weight", "offset_conv.bias", "offset"):
        assert_bf16_close(g[k], rg[k], k)


def test_bf16_config4_full_size_every_tensor(gpu_handle):
    """BASELINE config 4 per GPU (B=64, C=O=256, 28x28, bf16) at full size: every tensor
    against the C oracle run on the same bf16 inputs over the whole batch — the outputs
    from the oracle's own fp32 offsets (sampling is continuous in position, so the bf16
    rounding of the offsets, ~4e-3 px, stays inside the tolerance), the backward
    conditioned on the device's bf16 offsets (knife edges), and the four parameter
    gradients as 50,176-pixel reductions."""
    bits, v, s = _case(11, B=64, C=256, O_=256, H=28, W=28)
    out, off, g = _device(gpu_handle, bits, s)
    assert np.isfinite(out).all() and all(np.isfinite(t).all() for t in g.values())
    desc = R.make_desc((64, 256, 28, 28), v["w"].shape, (1, 1), (1, 1))
    ro, roff = R.forward(desc, v["x"], v["w_off"], v["b_off"], v["w"], v["b"])
    rg = R.backward(desc, v["x"], off, v["w_off"], v["w"], v["grad_out"])
    # out: elementwise against the oracle sampling at the device's own (bf16-rounded)
    # offsets; against the oracle's fp32 offsets (~4e-3 px apart) only in max-norm, since
    # a sample moved by the offset rounding legitimately changes single elements by more
    # than a bf16 ulp (r03: one of 12.8M elements by 0.034·rms)
    ro_dev = R.forward_from_offsets(desc, v["x"], off, v["w"], v["b"])
    worst = {"out": assert_bf16_close(out, ro_dev, "out"),
             "offset_values": assert_bf16_close(off, roff, "offset values")}
    assert rel_err(out, ro) <= BF16_TOL, "out vs the oracle's own offsets (max-norm)"
    for k in ("x", "offset", "weight", "bias", "offset_conv.weight", "offset_conv.bias"):
        worst[k] = assert_bf16_close(g[k], rg[k], k)
    print("config 4 worst |Δ|/bound per tensor:", {k: round(v_, 3) for k, v_ in worst.items()})


def test_bf16_config4_full_size_bitwise_reproducible(gpu_handle):
    """BASELINE config 4 per GPU at full size, forward + backward twice in one process: every
    output bit for bit equal (the removed fused forward differed run to run
    here; the shipped schedule has no float atomics and fixed summation orders)."""
    bits, _, s = _case(12, B=64, C=256, O_=256, H=28, W=28, off_scale=1.5)
    r1 = _device(gpu_handle, bits, s)
    r2 = _device(gpu_handle, bits, s)
    np.testing.assert_array_equal(r1[0].view(np.uint32), r2[0].view(np.uint32), err_msg="out")
    np.testing.assert_array_equal(r1[1].view(np.uint32), r2[1].view(np.uint32), err_msg="off")
    for k in r1[2]:
        np.testing.assert_array_equal(r1[2][k].view(np.uint32), r2[2][k].view(np.uint32),
                                      err_msg=k)


@pytest.mark.parametrize("B,H,W", [(4, 20, 19), (24, 28, 28), (64, 28, 28)])
def test_bf16_dcol_kernel_vs_vendor_gemm(gpu_handle, monkeypatch, B, H, W):
    """The ∂columns of dcol_bf16 (short-K streaming kernel) against the vendor GEMM's on the
    same inputs (a handle created with DCN_DCOL_GEMM=1): every downstream tensor within the
    bf16 bound of the other, and the forward tensors bit for bit (the kernel is backward
    only). Both sum the same 256 exact bf16 products in fp32, in different orders, then
    round to bf16 once, so ∂col elements may differ by an ulp; ∂x / ∂offset sum them.
    Geometries: 1,520 pixels = 48 tiles of 32 in 24 ranges (one tile per wave);
    B = 24 at 28x28, 21 tiles per range (3 or 2 per wave: the second register set and the odd
    tail); config 4 itself (56 per range, 7 per wave). C = 512 (18 row groups) is outside
    DCN_BF16 (C <= 256), so no op reaches it."""
    bits, _, s = _case(13, B=B, C=256, O_=256, H=H, W=W, off_scale=1.5)
    a = _device(gpu_handle, bits, s)
    monkeypatch.setenv("DCN_DCOL_GEMM", "1")
    h2 = rt.Handle(0)
    try:
        b = _device(h2, bits, s)
    finally:
        h2.close()
    np.testing.assert_array_equal(a[0].view(np.uint32), b[0].view(np.uint32), err_msg="out")
    np.testing.assert_array_equal(a[1].view(np.uint32), b[1].view(np.uint32), err_msg="off")
    for k in ("x", "offset", "offset_conv.weight", "offset_conv.bias"):
        assert_bf16_close(a[2][k], b[2][k], k)
    for k in ("weight", "bias"):  # before the ∂columns: untouched
        np.testing.assert_array_equal(a[2][k].view(np.uint32), b[2][k].view(np.uint32),
                                      err_msg=k)


@pytest.mark.parametrize("B,H,W,k", [(3, 13, 13, (3, 3)), (5, 23, 23, (3, 3)),
                                     (24, 28, 28, (3, 3)), (64, 28, 28, (3, 3)),
                                     (2, 20, 20, (1, 1))])
def test_bf16_dw_stream_vs_vendor_gemm(gpu_handle, monkeypatch, B, H, W, k):
    """∂W of dw_stream_bf16 (split-K streaming MFMA kernel over the stored columns,
    csrc/dcn_dw_bf16.hip) against the vendor GEMM's (a handle created with DCN_DW_GEMM=1) on
    the same inputs, and against the oracle: both sum exact bf16 products in fp32 (different
    orders), so ∂W may differ by one bf16 rounding; every other tensor is untouched by the
    choice (bit for bit). Geometries: 507 pixels = 16 stages of 32 in 16 one-stage ranges (a
    27-pixel last stage: the masked tail); 2,645 pixels (a 21-pixel last stage); B = 24 at
    28x28 (28 ranges of 21 stages: the unrolled ring plus a one-stage tail); config 4 (56
    stages per range); a 1x1 kernel (K = 256: one column tile, 25 one-stage ranges)."""
    pad = (1, 1) if k == (3, 3) else (0, 0)
    bits, v, s = _case(17 + B, B=B, C=256, O_=256, H=H, W=W, off_scale=1.5, k=k, p=pad)
    a = _device(gpu_handle, bits, s, pad=pad)
    monkeypatch.setenv("DCN_DW_GEMM", "1")
    h2 = rt.Handle(0)
    try:
        b = _device(h2, bits, s, pad=pad)
    finally:
        h2.close()
    np.testing.assert_array_equal(a[0].view(np.uint32), b[0].view(np.uint32), err_msg="out")
    np.testing.assert_array_equal(a[1].view(np.uint32), b[1].view(np.uint32), err_msg="off")
    for name in ("x", "offset", "bias", "offset_conv.weight", "offset_conv.bias"):
        np.testing.assert_array_equal(a[2][name].view(np.uint32), b[2][name].view(np.uint32),
                                      err_msg=name)
    gw, gv = a[2]["weight"].astype(np.float64), b[2]["weight"].astype(np.float64)
    rms = float(np.sqrt(np.mean(gv * gv)))
    lim = 2.0 ** -7 * np.abs(gv) + 2.0 ** -14 * rms
    assert np.all(np.abs(gw - gv) <= lim), \
        f"∂W: {int((np.abs(gw - gv) > lim).sum())} elements past one bf16 rounding of the GEMM's"
    if B <= 5:
        _, _, cache = O.forward(v["x"], v["w_off"], v["b_off"], v["w"], v["b"], s, pad,
                                offsets=a[1])
        rg = O.backward(cache, v["grad_out"])
        assert_bf16_close(a[2]["weight"], rg["weight"], "∂W vs oracle")


@pytest.mark.parametrize("B,C,H,W,s", [(8, 256, 28, 28, (1, 1)), (3, 64, 20, 17, (1, 1)),
                                       (2, 32, 30, 26, (2, 2))])
def test_bf16_bins_one_block_sort_vs_chunked(gpu_handle, B, C, H, W, s):
    """K5's sample bins from one block radix sort per image (bins_sort_seg: H·W·9 <= 8192)
    against the chunked three-kernel sort (dcn_debug_bins_chunked): the same stable order and
    the same records, so every output tensor is bit for bit the same (deform_conv.py:47-52
    autodiff). Geometries: config 4's 28x28 (7,056 samples per image), ragged 20x17, and
    stride 2 (a 15x13 output over a 30x26 input)."""
    bits, _, st = _case(71, B=B, C=C, O_=64, H=H, W=W, s=s, off_scale=2.0)
    a = _device(gpu_handle, bits, st)
    rt.check(gpu_handle.lib.dcn_debug_bins_chunked(1))
    try:
        b = _device(gpu_handle, bits, st)
    finally:
        rt.check(gpu_handle.lib.dcn_debug_bins_chunked(0))
    np.testing.assert_array_equal(a[0].view(np.uint32), b[0].view(np.uint32), err_msg="out")
    for name in a[2]:
        np.testing.assert_array_equal(a[2][name].view(np.uint32), b[2][name].view(np.uint32),
                                      err_msg=name)


@pytest.mark.parametrize("k,pad,C,H,W", [((1, 3), (0, 1), 24, 13, 11), ((3, 1), (1, 0), 24, 13, 11),
                                         ((2, 2), (1, 1), 24, 13, 11),
                                         ((1, 3), (0, 1), 64, 9, 8), ((2, 2), (1, 1), 128, 6, 12)])
def test_bf16_nonsquare_kernels_vs_oracle(gpu_handle, k, pad, C, H, W):
    """kh*kw outside {1,4,6,9} takes the generic offset-conv backward, which reads the fp32
    copy of x that the forward left in the workspace (the layouts of dcn_forward and
    dcn_backward share that region): ∂W_off must match the oracle. With C % 64 == 0 the
    bf16 MFMA backward takes them instead (J = 6 and 8 offset channels: J8 padding)."""
    bits, v, s = _case(31, B=2, C=C, O_=16, H=H, W=W, k=k, p=pad)
    out, off, g = _device(gpu_handle, bits, s, pad=pad)
    ro, _, cache = O.forward(v["x"], v["w_off"], v["b_off"], v["w"], v["b"], s, pad,
                             offsets=off)
    rg = O.backward(cache, v["grad_out"])
    assert_bf16_close(out, ro, "out")
    for name in ("x", "weight", "bias", "offset_conv.weight", "offset_conv.bias", "offset"):
        assert_bf16_close(g[name], rg[name], name)


def test_bf16_backward_with_attached_comm_single_rank(gpu_handle):
    """dcn_set_comm on a 1-rank world: dcn_backward sums the fp32 working copies of the
    parameter gradients over the ranks (the identity here) on its comm stream and rounds
    them to bf16 there; every gradient must equal the run without a communicator."""
    import dcn_dp
    bits, v, s = _case(41, B=3, C=32, O_=24, H=15, W=14)
    ref = _device(gpu_handle, bits, s)
    comm = dcn_dp.RcclComm(gpu_handle, 1, 0, dcn_dp.RcclComm.unique_id())
    try:
        got = _device(gpu_handle, bits, s, comm=comm)
    finally:
        comm.close()
    np.testing.assert_array_equal(got[0], ref[0])
    for name in ref[2]:
        np.testing.assert_array_equal(got[2][name], ref[2][name], err_msg=name)



@pytest.mark.parametrize("C,H,W", [(256, 28, 28), (64, 20, 20), (192, 13, 16)])
def test_bf16_offset_conv_fold_vs_separate_transpose(gpu_handle, C, H, W):
    """f3: where it applies the bf16 offset conv stages its windows from the
    NCHW x and writes the channels-last xT itself (no transpose launch). Against the
    separate-transpose schedule (dcn_debug_force_generic also turns the fold off; both runs
    unfused, so their columns and GEMMs are the same): offsets and out bit for bit, which
    needs every xT element right, and the forward against the oracle."""
    bits, v, s = _case(71 + C, B=2, C=C, O_=64, H=H, W=W, off_scale=1.5)
    gpu_handle.set_fwd_path(rt.DCN_FWD_UNFUSED)
    try:
        out_a, off_a, _ = _device(gpu_handle, bits, s)
        rt.check(gpu_handle.lib.dcn_debug_force_generic(1))
        try:
            out_b, off_b, _ = _device(gpu_handle, bits, s)
        finally:
            rt.check(gpu_handle.lib.dcn_debug_force_generic(0))
    finally:
        gpu_handle.set_fwd_path(rt.DCN_FWD_AUTO)
    np.testing.assert_array_equal(off_a.view(np.uint32), off_b.view(np.uint32))
    np.testing.assert_array_equal(out_a.view(np.uint32), out_b.view(np.uint32))
    ro, _, _ = O.forward(v["x"], v["w_off"], v["b_off"], v["w"], v["b"], s, (1, 1), offsets=off_a)
    assert_bf16_close(out_a, ro, "out (fold)")


def test_bf16_fused_forward_with_attached_comm_single_rank(gpu_handle):
    """The config-4 data-parallel step on one rank: DCN_FWD_AUTO's fused bf16 forward (C=256,
    its columns stored for the backward) with the RCCL communicator attached — the overlapped
    gradient exchange must leave every tensor as the run without a communicator."""
    import dcn_dp
    bits, v, s = _case(43, B=4, C=256, O_=256, H=28, W=28)
    ref = _device(gpu_handle, bits, s)
    comm = dcn_dp.RcclComm(gpu_handle, 1, 0, dcn_dp.RcclComm.unique_id())
    try:
        got = _device(gpu_handle, bits, s, comm=comm)
    finally:
        comm.close()
    np.testing.assert_array_equal(got[0], ref[0])
    for name in ref[2]:
        np.testing.assert_array_equal(got[2][name], ref[2][name], err_msg=name)
