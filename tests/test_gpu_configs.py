"""GPU parity at the BASELINE.json geometries (configs 2, 3 and 5) against the oracles, and
the data-parallel exchange hooks (dcn_set_comm, dcn_set_grad_stream, dcn_allreduce_grads)
on a 1-rank world.

Oracles: oracle/dcn_ref.c (fp32 restatement of deform_conv.py:56-81 and its autodiff, the
four parameter reductions accumulated in double) over the WHOLE batch, and the float64
NumPy oracle where its size allows. Tolerances as in test_gpu_parity: elementwise
|Δ| <= 1e-4 + 1e-4·|ref|; reductions max|Δ|/max|ref| <= 1e-4. Parity is unpinned w.r.t.
Jittor itself; config 5's dilation / deform groups are extensions checked
against our own restatement only.
"""
import ctypes

import numpy as np
import pytest

import dcn_oracle as O
import dcn_runtime as rt
import ref_lib as R
from conftest import assert_close, assert_close_reduction
from test_gpu_parity import Dev, _device_fwd_bwd, _rand_case

pytestmark = pytest.mark.gpu

PARAMS = ("weight", "bias", "offset_conv.weight", "offset_conv.bias")


def _c_oracle_all(c, dev_off):
    """C oracle over the whole batch: forward from its own offsets, backward conditioned on
    the device's offsets (∂offset is discontinuous at integer sample coordinates)."""
    desc = R.make_desc(c["x"].shape, c["w"].shape, c["stride"], c["padding"], c["dil"], c["G"],
                       c["b"] is not None)
    ro, roff = R.forward(desc, c["x"], c["w_off"], c["b_off"], c["w"], c["b"])
    rg = R.backward(desc, c["x"], dev_off, c["w_off"], c["w"], c["grad_out"])
    return ro, roff, rg


def _check_all(out, off, g, ro, roff, rg, what):
    assert_close(out, ro, what=f"{what} out")
    assert_close(off, roff, what=f"{what} offset")
    assert_close(g["x"], rg["x"], what=f"{what} ∂x")
    assert_close(g["offset"], rg["offset"], what=f"{what} ∂offset")
    for k in PARAMS:
        if k in rg:
            assert_close_reduction(g[k], rg[k], what=f"{what} ∂{k}")


def _device_forward_only(h, c, fwd_path=rt.DCN_FWD_AUTO):
    """dcn_forward alone with the forward-only workspace (config 2 is forward-only)."""
    x, wo, bo, w, b = c["x"], c["w_off"], c["b_off"], c["w"], c["b"]
    B, C, H, W = x.shape
    O_, _, kh, kw = w.shape
    desc = rt.make_desc(B, C, H, W, O_, (kh, kw), c["stride"], c["padding"], c["dil"], c["G"],
                        bias=b is not None)
    Ho, Wo = rt.out_shape(desc)
    J = wo.shape[0]
    D = Dev(h)
    vp = ctypes.c_void_p
    try:
        px, pwo, pbo, pw = D.up(x), D.up(wo), D.up(bo), D.up(w)
        pb = D.up(b) if b is not None else None
        pout, poff = D.zeros(B * O_ * Ho * Wo * 4), D.zeros(B * J * Ho * Wo * 4)
        wsb = rt.workspace_bytes(desc, False)
        ws = D.zeros(wsb)
        h.set_fwd_path(fwd_path)
        rt.check(h.lib.dcn_forward(h.h, desc, vp(px), vp(pwo), vp(pbo), vp(pw), vp(pb), vp(pout),
                                   vp(poff), vp(ws), wsb), "dcn_forward")
        return D.down(pout, (B, O_, Ho, Wo)), D.down(poff, (B, J, Ho, Wo))
    finally:
        h.set_fwd_path(rt.DCN_FWD_AUTO)
        D.free()


# ---- config 2: B=8, 64 -> 128, 56x56, k3 s1 p1, fp32, forward only ----------------------

@pytest.mark.parametrize("fwd_path", [rt.DCN_FWD_AUTO, rt.DCN_FWD_UNFUSED, rt.DCN_FWD_FUSED])
def test_config2_forward_vs_float64_oracle(gpu_handle, fwd_path):
    """BASELINE config 2 at its geometry through every forward schedule, against the
    float64 NumPy oracle (offsets from its own conv; the rest conditioned on the device's
    offsets only to keep the comparison about sampling + GEMM)."""
    c = _rand_case(202, B=8, C=64, O_=128, H=56, W=56)
    out, off = _device_forward_only(gpu_handle, c, fwd_path)
    _, roff, _ = O.forward(c["x"], c["w_off"], c["b_off"], c["w"], c["b"], c["stride"],
                           c["padding"])
    assert_close(off, roff, what="config2 offset")
    ro, _, _ = O.forward(c["x"], c["w_off"], c["b_off"], c["w"], c["b"], c["stride"],
                         c["padding"], offsets=off)
    assert_close(out, ro, what=f"config2 out (path {fwd_path})")


def test_config2_host_api_vs_c_oracle(gpu_handle):
    """Config 2 through the host-pointer API (the NumPy / Jittor caller's path)."""
    from deform_conv import dcn_forward_numpy
    c = _rand_case(203, B=8, C=64, O_=128, H=56, W=56)
    out, off = dcn_forward_numpy(c["x"], c["w_off"], c["b_off"], c["w"], c["b"], c["stride"],
                                 c["padding"], handle=gpu_handle)
    desc = R.make_desc(c["x"].shape, c["w"].shape, c["stride"], c["padding"])
    ro, roff = R.forward(desc, c["x"], c["w_off"], c["b_off"], c["w"], c["b"])
    assert_close(off, roff, what="config2 host offset")
    assert_close(out, ro, what="config2 host out")


# ---- config 3: B=64, C=O=256, 56x56, k3 s1 p1, fp32 fwd+bwd (the metric's workload) --------

def test_config3_full_batch_every_tensor_vs_c_oracle(gpu_handle):
    """BASELINE config 3 at full size: out, offsets, ∂x, ∂offset for all 64 images and the
    four parameter gradients (sums over 200,704 pixels, incl. the side-stream partial sums
    and tile folds of the device path) against the C oracle over the whole batch."""
    c = _rand_case(61, B=64, C=256, O_=256, H=56, W=56)
    out, off, g = _device_fwd_bwd(gpu_handle, c)
    ro, roff, rg = _c_oracle_all(c, off)
    _check_all(out, off, g, ro, roff, rg, "config3")
    # the host-pointer path on a module's state: auto image chunks (205 MB of x -> 4), the
    # transfers pipelined with the kernels, the backward reusing each chunk's columns
    from deform_conv import dcn_backward_numpy, dcn_forward_numpy
    st = rt.HostState(gpu_handle)
    hout, hoff, ctx = dcn_forward_numpy(c["x"], c["w_off"], c["b_off"], c["w"], c["b"],
                                        c["stride"], c["padding"], state=st, return_ctx=True)
    # the per-image offset conv does not depend on how the batch is cut
    np.testing.assert_array_equal(hoff, off, err_msg="config3 host offsets")
    hg = dcn_backward_numpy(c["x"], hoff, c["w_off"], c["w"], True, c["grad_out"], c["stride"],
                            c["padding"], ctx=ctx)
    st.close()
    _check_all(hout, hoff, hg, ro, roff, rg, "config3 host (chunked)")


def test_config3_full_size_bitwise_reproducible(gpu_handle):
    """Config 3 at full size, forward + backward twice in one process: every output bit for
    bit equal (no float atomics; bins ordered by sample index; fixed-order partial sums)."""
    c = _rand_case(62, B=64, C=256, O_=256, H=56, W=56, off_scale=1.5)
    r1 = _device_fwd_bwd(gpu_handle, c)
    r2 = _device_fwd_bwd(gpu_handle, c)
    np.testing.assert_array_equal(r1[0].view(np.uint32), r2[0].view(np.uint32), err_msg="out")
    np.testing.assert_array_equal(r1[1].view(np.uint32), r2[1].view(np.uint32), err_msg="off")
    for k in r1[2]:
        np.testing.assert_array_equal(r1[2][k].view(np.uint32), r2[2][k].view(np.uint32),
                                      err_msg=k)


# ---- config 5: B=64, C=O=512, 14x14, k3 s2 p1, dilation 2, deform_groups 4 ----------------

def test_config5_full_batch_every_tensor_vs_c_oracle(gpu_handle):
    """BASELINE config 5 (the DCNv1 option set: C > 256 and 4 deform groups take the
    unfused channels-last / generic kernels) at full size against the C oracle over the
    whole batch. Extension semantics: parity against our own restatement."""
    c = _rand_case(505, B=64, C=512, O_=512, H=14, W=14, s=(2, 2), p=(1, 1), dil=(2, 2), G=4)
    out, off, g = _device_fwd_bwd(gpu_handle, c)
    assert out.shape == (64, 512, 6, 6) and off.shape == (64, 72, 6, 6)
    ro, roff, rg = _c_oracle_all(c, off)
    _check_all(out, off, g, ro, roff, rg, "config5")


def test_config5_two_images_vs_float64_oracle(gpu_handle):
    """Config 5's geometry on two images against the independent float64 NumPy oracle."""
    c = _rand_case(506, B=2, C=512, O_=512, H=14, W=14, s=(2, 2), p=(1, 1), dil=(2, 2), G=4)
    out, off, g = _device_fwd_bwd(gpu_handle, c)
    _, roff, _ = O.forward(c["x"], c["w_off"], c["b_off"], c["w"], c["b"], c["stride"],
                           c["padding"], c["dil"], c["G"])
    ro, _, cache = O.forward(c["x"], c["w_off"], c["b_off"], c["w"], c["b"], c["stride"],
                             c["padding"], c["dil"], c["G"], offsets=off)
    _check_all(out, off, g, ro, roff, O.backward(cache, c["grad_out"]), "config5 f64")


@pytest.mark.parametrize("geo", [
    dict(C=512, O_=64, H=14, W=14, s=(2, 2), p=(1, 1), dil=(2, 2), G=4),  # config 5's offset conv
    dict(C=64, O_=32, H=13, W=11, s=(2, 1), p=(1, 0), dil=(1, 2), G=1),   # ragged, mixed s / dil
])
def test_offset_conv_gemm_vs_valu_kernels(gpu_handle, geo):
    """r05: the fp32 offset conv of geometries without an MFMA offset-conv kernel runs as GEMMs
    over its own im2col (dcn_api.cpp offset_conv_fwd_gemm / _bwd_gemm). Same results as the
    VALU kernels it replaced (dcn_debug_offset_gemm(0)) up to fp32 summation order, and the
    whole step against the C oracle (conditioned on the device's offsets)."""
    c = _rand_case(511, B=4, **geo)
    L = gpu_handle.lib
    rt.check(L.dcn_debug_offset_gemm(0))
    try:
        out0, off0, g0 = _device_fwd_bwd(gpu_handle, c)
    finally:
        rt.check(L.dcn_debug_offset_gemm(1))
    out1, off1, g1 = _device_fwd_bwd(gpu_handle, c)
    assert_close(off1, off0, what="offsets: GEMM vs VALU")
    for k in ("offset_conv.weight", "offset_conv.bias"):
        assert_close_reduction(g1[k], g0[k], what=f"∂{k}: GEMM vs VALU")
    ro, roff, rg = _c_oracle_all(c, off1)
    _check_all(out1, off1, g1, ro, roff, rg, "offset-conv GEMM path")


def _bitwise_equal(r1, r0, what):
    np.testing.assert_array_equal(r1[0].view(np.uint32), r0[0].view(np.uint32), err_msg=f"{what} out")
    np.testing.assert_array_equal(r1[1].view(np.uint32), r0[1].view(np.uint32), err_msg=f"{what} off")
    for k in r0[2]:
        np.testing.assert_array_equal(r1[2][k].view(np.uint32), r0[2][k].view(np.uint32),
                                      err_msg=f"{what} {k}")


def test_offset_conv_gemm_backward_reuses_forward_im2col(gpu_handle):
    """r06: on the offset-conv GEMM route the forward keeps its offset-conv im2col (and W') in
    the workspace, and a DCN_BWD_COL_IN_WS backward reads them instead of recomputing. A
    backward without the flag recomputes everything: every output bit for bit the same. A
    forward that took the VALU offset conv (dcn_debug_offset_gemm(0)) leaves no im2col, and
    the handle's per-workspace record makes the GEMM-route backward after it recompute: the
    gradients stay the oracle's."""
    c = _rand_case(513, B=4, C=512, O_=64, H=14, W=14, s=(2, 2), p=(1, 1), dil=(2, 2), G=4)
    h = gpu_handle
    r1 = _device_fwd_bwd(h, c)
    r0 = _device_fwd_bwd(h, c, bwd_flags=0)
    _bitwise_equal(r1, r0, "reuse vs recompute")
    L = h.lib
    rt.check(L.dcn_debug_offset_gemm(0))
    try:
        out, off, g = _device_fwd_bwd(h, c, between=lambda: rt.check(L.dcn_debug_offset_gemm(1)))
    finally:
        rt.check(L.dcn_debug_offset_gemm(1))
    ro, roff, rg = _c_oracle_all(c, off)
    _check_all(out, off, g, ro, roff, rg, "VALU forward, GEMM-route backward")


@pytest.mark.parametrize("math", [3, 6])
def test_offset_conv_gemm_native_under_split_math(gpu_handle, math):
    """dcn_set_math covers the op's three GEMMs only (include/dcn.h). The offset
    conv's own GEMMs (ocg path: stride / dilation != 1) stay native f32 under every math mode,
    so the offsets are bit for bit the native-mode ones (the gradients are not: ∂col is one of
    the three GEMMs)."""
    c = _rand_case(512, B=4, C=512, O_=64, H=14, W=14, s=(2, 2), p=(1, 1), dil=(2, 2), G=4)
    h = gpu_handle
    _, off0, _ = _device_fwd_bwd(h, c)
    h.set_math(math)
    try:
        _, off1, _ = _device_fwd_bwd(h, c)
    finally:
        h.set_math(0)
    np.testing.assert_array_equal(off1, off0, err_msg=f"offsets under dcn_set_math({math})")


# ---- data-parallel exchange hooks on one rank -------------------------------------------

def test_fp32_backward_with_attached_comm_single_rank(gpu_handle):
    """dcn_set_comm on a 1-rank world: the in-backward all-reduce (∂W/∂b on the comm stream
    beside the rest of the backward, ∂W_off/∂b_off at the end) is the identity, and the
    handle's stream waits for it: every gradient equals the run without a communicator."""
    import dcn_dp
    h = gpu_handle
    c = _rand_case(77, B=3, C=64, O_=32, H=21, W=19)
    ref = _device_fwd_bwd(h, c)
    comm = dcn_dp.RcclComm(h, 1, 0, dcn_dp.RcclComm.unique_id())
    try:
        h.set_comm(comm)
        got = _device_fwd_bwd(h, c)
    finally:
        h.set_comm(None)
        comm.close()
    for k in ref[2]:
        np.testing.assert_array_equal(got[2][k], ref[2][k], err_msg=k)


def test_grad_stream_is_released_when_dw_is_final(gpu_handle):
    """dcn_set_grad_stream: a copy of ∂W/∂b enqueued on the released stream right after
    dcn_backward returns (what bench.py's torch all-reduce does) sees the final values."""
    import torch
    h = gpu_handle
    dev = torch.device("cuda", 0)
    c = _rand_case(78, B=4, C=128, O_=64, H=28, W=28)
    x, wo, bo, w, b, gout = (torch.from_numpy(c[k]).to(dev) for k in
                             ("x", "w_off", "b_off", "w", "b", "grad_out"))
    B, C, H, W = x.shape
    O_ = w.shape[0]
    desc = rt.make_desc(B, C, H, W, O_, (3, 3), (1, 1), (1, 1))
    Ho, Wo = rt.out_shape(desc)
    out = torch.empty(B, O_, Ho, Wo, device=dev)
    off = torch.empty(B, 18, Ho, Wo, device=dev)
    gx, gw, gb = torch.empty_like(x), torch.empty_like(w), torch.empty_like(b)
    gwo, gbo, goff = torch.empty_like(wo), torch.empty_like(bo), torch.empty_like(off)
    wsb = rt.workspace_bytes(desc, True)
    ws = torch.empty(wsb, dtype=torch.uint8, device=dev)
    main = torch.cuda.current_stream(dev)
    gs = torch.cuda.Stream(dev)
    P = lambda t: t.data_ptr()
    L = h.lib
    h.set_stream(main.cuda_stream)
    try:
        h.set_grad_stream(gs.cuda_stream)
        rt.check(L.dcn_forward(h.h, desc, P(x), P(wo), P(bo), P(w), P(b), P(out), P(off),
                               P(ws), wsb))
        rt.check(L.dcn_backward(h.h, desc, P(x), P(off), P(wo), P(w), P(gout), P(gx), P(gw),
                                P(gb), P(gwo), P(gbo), P(goff), P(ws), wsb, rt.DCN_BWD_COL_IN_WS))
        with torch.cuda.stream(gs):
            gw_seen, gb_seen = gw.clone(), gb.clone()
        main.wait_stream(gs)
        torch.cuda.synchronize(dev)
    finally:
        h.set_grad_stream(None)
        h.use_own_stream()
    assert torch.equal(gw_seen, gw) and torch.equal(gb_seen, gb)
    rg = R.backward(R.make_desc(c["x"].shape, c["w"].shape, (1, 1), (1, 1)), c["x"],
                    off.cpu().numpy(), c["w_off"], c["w"], c["grad_out"])
    assert_close_reduction(gw_seen.cpu().numpy(), rg["weight"], what="∂W on the grad stream")
    assert_close_reduction(gb_seen.cpu().numpy(), rg["bias"], what="∂b on the grad stream")


def test_allreduce_grads_bf16_and_overrun_rejected(gpu_handle):
    """dcn_allreduce_grads with a dtype: a bf16 buffer reduces in bf16 (identity on one
    rank); a count that runs past the buffer's allocation is rejected before RCCL runs."""
    import dcn_dp
    h = gpu_handle
    comm = dcn_dp.RcclComm(h, 1, 0, dcn_dp.RcclComm.unique_id())
    n = 631_570
    p = h.malloc(n * 2)
    try:
        bits = np.random.default_rng(5).integers(0x3000, 0x4000, n).astype(np.uint16)
        rt.check(h.lib.dcn_memcpy_h2d(h.h, ctypes.c_void_p(p), bits.ctypes.data_as(ctypes.c_void_p),
                                      bits.nbytes))
        comm.allreduce(p, n, rt.DCN_BF16)
        back = np.empty_like(bits)
        h.synchronize()
        rt.check(h.lib.dcn_memcpy_d2h(h.h, back.ctypes.data_as(ctypes.c_void_p), ctypes.c_void_p(p),
                                      back.nbytes))
        np.testing.assert_array_equal(back, bits)
        with pytest.raises(RuntimeError, match="past the end"):
            comm.allreduce(p, n, rt.DCN_F32)  # n fp32 values = 2x the bf16 buffer
        with pytest.raises(RuntimeError, match="dtype"):
            comm.allreduce(p, n, 7)
    finally:
        h.free(p)
        comm.close()
