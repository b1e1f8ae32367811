"""The host-pointer API (dcn_forward_host / dcn_backward_host[_ex]): the NumPy / Jittor-CPU
caller's path (train.py:408-414 through the module), on libdcn.

Pinned here:
  * staged transfers (pinned ring, host copy threads) move every byte: results equal the
    oracle, also with a chunk size that splits every tensor into ragged pieces;
  * DCN_HOST_REUSE_FWD (the backward reusing its forward's device copies and columns) gives
    bitwise the gradients of a backward that uploads and recomputes everything;
  * reuse is refused (DCN_ERR_INVALID) for arrays that are not the forward's, and the Python
    shim falls back to a full upload when another host call ran in between (two layers);
  * per-module host states (dcn_host_state): four stacked modules on one handle each reuse
    their own forward (the library accepts DCN_HOST_REUSE_FWD for all four backwards);
  * the image-chunk transfer pipeline: ragged chunk counts match the oracle, reuse equals
    the full upload bitwise per chunk plan, and runs are bitwise reproducible.
"""
import ctypes
import os

import numpy as np
import pytest

import dcn_oracle as O
import dcn_runtime as rt
from conftest import assert_close, assert_close_reduction
from deform_conv import DeformConv2dNumpy, dcn_backward_numpy, dcn_forward_numpy

pytestmark = pytest.mark.gpu


def _case(seed, B=2, C=16, O_=12, H=13, W=11, s=(1, 1)):
    rng = np.random.default_rng(seed)
    x = rng.standard_normal((B, C, H, W)).astype(np.float32)
    wo = (rng.standard_normal((18, C, 3, 3)) / np.sqrt(C * 9)).astype(np.float32)
    bo = rng.uniform(-0.5, 0.5, 18).astype(np.float32)
    w = (rng.standard_normal((O_, C, 3, 3)) * np.sqrt(2 / (C * 9))).astype(np.float32)
    b = (rng.standard_normal(O_) * 0.1).astype(np.float32)
    Ho, Wo = O.out_size(H, W, 3, 3, *s, 1, 1, 1, 1)
    gout = rng.standard_normal((B, O_, Ho, Wo)).astype(np.float32)
    return x, wo, bo, w, b, gout, s


def _grads_equal(a, b):
    assert a.keys() == b.keys()
    for k in a:
        np.testing.assert_array_equal(a[k], b[k], err_msg=k)


def test_host_reuse_bitwise_equals_full_upload():
    h = rt.Handle(0)
    x, wo, bo, w, b, gout, s = _case(1)
    out, off, ctx = dcn_forward_numpy(x, wo, bo, w, b, s, (1, 1), handle=h, return_ctx=True)
    g_reuse = dcn_backward_numpy(x, off, wo, w, True, gout, s, (1, 1), handle=h, ctx=ctx)
    g_full = dcn_backward_numpy(x, off, wo, w, True, gout, s, (1, 1), handle=h)
    _grads_equal(g_reuse, g_full)
    ro, roff, cache = O.forward(x, wo, bo, w, b, s, (1, 1))
    assert_close(out, ro, what="out")
    _, _, cache = O.forward(x, wo, bo, w, b, s, (1, 1), offsets=off)
    rg = O.backward(cache, gout)
    assert_close(g_reuse["x"], rg["x"], what="∂x")
    for k in ("weight", "bias", "offset_conv.weight", "offset_conv.bias"):
        assert_close_reduction(g_reuse[k], rg[k], what=k)
    h.close()


def test_host_reuse_refused_for_other_arrays():
    h = rt.Handle(0)
    x, wo, bo, w, b, gout, s = _case(2)
    out, off = dcn_forward_numpy(x, wo, bo, w, b, s, (1, 1), handle=h)
    desc = rt.make_desc(*x.shape, w.shape[0], (3, 3), s, (1, 1), bias=True)
    x2 = x.copy()  # same values, another array: the library cannot vouch for it
    bufs = [np.empty_like(x), np.empty_like(w), np.empty(w.shape[0], np.float32),
            np.empty_like(wo), np.empty(18, np.float32), np.empty_like(off)]
    r = h.lib.dcn_backward_host_ex(h.h, desc, rt.ptr(x2), rt.ptr(off), rt.ptr(wo), rt.ptr(w),
                                   rt.ptr(gout), *[rt.ptr(a) for a in bufs], rt.HOST_REUSE_FWD)
    assert r == -1  # DCN_ERR_INVALID
    assert b"DCN_HOST_REUSE_FWD" in h.lib.dcn_last_error()
    # the same call on the forward's own arrays is accepted
    r = h.lib.dcn_backward_host_ex(h.h, desc, rt.ptr(x), rt.ptr(off), rt.ptr(wo), rt.ptr(w),
                                   rt.ptr(gout), *[rt.ptr(a) for a in bufs], rt.HOST_REUSE_FWD)
    assert r == 0
    # ... once: the backward consumed the forward's columns
    r = h.lib.dcn_backward_host_ex(h.h, desc, rt.ptr(x), rt.ptr(off), rt.ptr(wo), rt.ptr(w),
                                   rt.ptr(gout), *[rt.ptr(a) for a in bufs], rt.HOST_REUSE_FWD)
    assert r == -1
    h.close()


def test_two_layers_share_a_handle():
    """Layer 1's backward runs after layer 2's forward and backward: its context is stale, so
    the shim uploads again (no reuse) and the gradients stay right."""
    h = rt.Handle(0)
    x, wo, bo, w, b, gout, s = _case(3)
    x2, wo2, bo2, w2, b2, gout2, _ = _case(4)
    out1, off1, c1 = dcn_forward_numpy(x, wo, bo, w, b, s, (1, 1), handle=h, return_ctx=True)
    out2, off2, c2 = dcn_forward_numpy(x2, wo2, bo2, w2, b2, s, (1, 1), handle=h, return_ctx=True)
    assert not c1.matches(h, x, wo, w, off1) and c2.matches(h, x2, wo2, w2, off2)
    g2 = dcn_backward_numpy(x2, off2, wo2, w2, True, gout2, s, (1, 1), handle=h, ctx=c2)
    g1 = dcn_backward_numpy(x, off1, wo, w, True, gout, s, (1, 1), handle=h, ctx=c1)
    g1_ref = dcn_backward_numpy(x, off1, wo, w, True, gout, s, (1, 1), handle=h)
    _grads_equal(g1, g1_ref)
    g2_ref = dcn_backward_numpy(x2, off2, wo2, w2, True, gout2, s, (1, 1), handle=h)
    _grads_equal(g2, g2_ref)
    h.close()


def test_module_backward_reuses_forward():
    m = DeformConv2dNumpy(16, 12, 3, 1, 1, seed=5)
    rng = np.random.default_rng(5)
    m.offset_conv.weight[...] = rng.standard_normal(m.offset_conv.weight.shape) * 0.05
    x = rng.standard_normal((2, 16, 10, 12)).astype(np.float32)
    out = m(x)
    gout = rng.standard_normal(out.shape).astype(np.float32)
    gx = m.backward(gout)
    _, _, cache = O.forward(x, m.offset_conv.weight, m.offset_conv.bias, m.weight, m.bias,
                            (1, 1), (1, 1), offsets=m._ctx[1])
    rg = O.backward(cache, gout)
    assert_close(gx, rg["x"], what="module ∂x")
    assert_close_reduction(m.weight.grad, rg["weight"], what="module ∂W")


@pytest.mark.parametrize("chunk_mb,threads", [(1, 3), (1, 1)])
def test_staging_ragged_chunks(monkeypatch, chunk_mb, threads):
    """Pinned staging (DCN_HOST_STAGING=1) with 1-MiB chunks and 1 or 3 copy threads: x
    (2.4 MiB), out, ∂x all split into ragged pieces; results equal the direct transfers'."""
    x, wo, bo, w, b, gout, s = _case(6, B=3, C=32, O_=24, H=61, W=109, s=(1, 1))
    h0 = rt.Handle(0)
    out0, off0 = dcn_forward_numpy(x, wo, bo, w, b, s, (1, 1), handle=h0)
    g0 = dcn_backward_numpy(x, off0, wo, w, True, gout, s, (1, 1), handle=h0)
    h0.close()
    monkeypatch.setenv("DCN_HOST_STAGING", "1")
    monkeypatch.setenv("DCN_HOST_CHUNK_MB", str(chunk_mb))
    monkeypatch.setenv("DCN_HOST_THREADS", str(threads))
    h = rt.Handle(0)  # staging is created with the handle's first host transfer
    out, off, ctx = dcn_forward_numpy(x, wo, bo, w, b, s, (1, 1), handle=h, return_ctx=True)
    g = dcn_backward_numpy(x, off, wo, w, True, gout, s, (1, 1), handle=h, ctx=ctx)
    g_full = dcn_backward_numpy(x, off, wo, w, True, gout, s, (1, 1), handle=h)
    _grads_equal(g, g_full)  # same handle: bitwise
    # across handles each GEMM engine autotunes on its own (timing-based), so the GEMM
    # summation orders may differ: fp32 rounding, not bits
    assert_close(out, out0, what="out")
    np.testing.assert_array_equal(off, off0)  # the offset conv has no autotuned GEMM
    assert_close(g["x"], g0["x"], what="∂x")
    for k in ("weight", "bias", "offset_conv.weight", "offset_conv.bias"):
        assert_close_reduction(g[k], g0[k], what=k)
    h.close()


def _spy_backward_flags(monkeypatch):
    lib = rt.load()
    calls, real = [], lib.dcn_backward_host_s

    def spy(*a):
        calls.append(a[-1])
        return real(*a)

    monkeypatch.setattr(lib, "dcn_backward_host_s", spy)
    return calls


def test_four_stacked_modules_each_reuse_their_forward(monkeypatch):
    """train.py:304-318 stacks four DeformConv2d on one handle and runs all forwards before
    any backward (optimizer.backward, :414). Each module keeps its own host state, so every
    backward reuses its own forward's columns: the library accepts DCN_HOST_REUSE_FWD for
    all four (it refuses the flag otherwise), and each module's grads match the oracle."""
    calls = _spy_backward_flags(monkeypatch)
    rng = np.random.default_rng(21)
    shapes = [(8, 12, 1), (12, 16, 2), (16, 16, 1), (16, 8, 1)]  # (C_in, C_out, stride)
    mods = []
    for i, (ci, co, st) in enumerate(shapes):
        m = DeformConv2dNumpy(ci, co, 3, st, 1, seed=30 + i)
        m.offset_conv.weight[...] = rng.standard_normal(m.offset_conv.weight.shape) * 0.1
        m.offset_conv.bias[...] = rng.uniform(-1, 1, m.offset_conv.bias.shape)
        mods.append(m)
    xs = [rng.standard_normal((2, 8, 17, 15)).astype(np.float32)]
    for m in mods:
        xs.append(m(xs[-1]))
    gins = [rng.standard_normal(xs[-1].shape).astype(np.float32)]
    for m in reversed(mods):
        gins.append(m.backward(gins[-1]))
    assert calls == [rt.HOST_REUSE_FWD] * 4
    assert len({id(m._hstate) for m in mods}) == 4
    for i, m in enumerate(mods):
        gout = gins[len(mods) - 1 - i]
        ro, _, _ = O.forward(xs[i], m.offset_conv.weight, m.offset_conv.bias, m.weight, m.bias,
                             m.stride, m.padding)
        assert_close(xs[i + 1], ro, what=f"module {i} out")
        _, _, cache = O.forward(xs[i], m.offset_conv.weight, m.offset_conv.bias, m.weight,
                                m.bias, m.stride, m.padding, offsets=m._ctx[1])
        rg = O.backward(cache, gout)
        assert_close(gins[len(mods) - i], rg["x"], what=f"module {i} ∂x")
        for k in ("weight", "bias", "offset_conv.weight", "offset_conv.bias"):
            p = m.bias if k == "bias" else (
                m.weight if k == "weight" else getattr(m.offset_conv, k.split(".")[1]))
            assert_close_reduction(p.grad, rg[k], what=f"module {i} ∂{k}")


@pytest.mark.parametrize("chunks", [1, 2, 3, 5])
def test_host_chunk_pipeline(chunks):
    """B = 5 cut into 1, 2 (2+3), 3 (1+2+2) or 5 image chunks: out / offsets / every gradient
    match the oracle; the reusing backward equals the full-upload backward bitwise (same
    chunk plan); a second run is bitwise the first."""
    x, wo, bo, w, b, gout, s = _case(40, B=5, C=16, O_=12, H=13, W=11)
    h = rt.Handle(0)
    st = rt.HostState(h, chunks)

    def run():
        out, off, ctx = dcn_forward_numpy(x, wo, bo, w, b, s, (1, 1), state=st, return_ctx=True)
        g = dcn_backward_numpy(x, off, wo, w, True, gout, s, (1, 1), ctx=ctx)
        return out, off, g

    out, off, g = run()
    g_full = dcn_backward_numpy(x, off, wo, w, True, gout, s, (1, 1), state=st)
    _grads_equal(g, g_full)
    out2, off2, g2 = run()
    np.testing.assert_array_equal(out, out2)
    np.testing.assert_array_equal(off, off2)
    _grads_equal(g, g2)
    ro, roff, _ = O.forward(x, wo, bo, w, b, s, (1, 1))
    assert_close(out, ro, what=f"out ({chunks} chunks)")
    assert_close(off, roff, what=f"offsets ({chunks} chunks)")
    _, _, cache = O.forward(x, wo, bo, w, b, s, (1, 1), offsets=off)
    rg = O.backward(cache, gout)
    assert_close(g["x"], rg["x"], what="∂x")
    assert_close(g["offset"], rg["offset"], what="∂offset")
    for k in ("weight", "bias", "offset_conv.weight", "offset_conv.bias"):
        assert_close_reduction(g[k], rg[k], what=f"∂{k} ({chunks} chunks)")
    st.close()
    h.close()


def test_host_state_rules():
    """A state refuses a reusing backward after another forward on it and a full backward
    without offsets, and outlives its handle only as an object to destroy."""
    x, wo, bo, w, b, gout, s = _case(41)
    h = rt.Handle(0)
    st = rt.HostState(h)
    out, off, ctx = dcn_forward_numpy(x, wo, bo, w, b, s, (1, 1), state=st, return_ctx=True)
    desc = rt.make_desc(*x.shape, w.shape[0], (3, 3), s, (1, 1), bias=True)
    bufs = [np.empty_like(x), np.empty_like(w), np.empty(w.shape[0], np.float32),
            np.empty_like(wo), np.empty(18, np.float32), None]
    r = h.lib.dcn_backward_host_s(st.s, desc, rt.ptr(x), None, rt.ptr(wo), rt.ptr(w),
                                  rt.ptr(gout), *[rt.ptr(a) for a in bufs], 0)
    assert r == -1 and b"off is required" in h.lib.dcn_last_error()
    x2 = x + 1
    dcn_forward_numpy(x2, wo, bo, w, b, s, (1, 1), state=st)
    r = h.lib.dcn_backward_host_s(st.s, desc, rt.ptr(x), rt.ptr(off), rt.ptr(wo), rt.ptr(w),
                                  rt.ptr(gout), *[rt.ptr(a) for a in bufs], rt.HOST_REUSE_FWD)
    assert r == -1 and b"DCN_HOST_REUSE_FWD" in h.lib.dcn_last_error()
    h.close()
    with pytest.raises(RuntimeError, match="destroyed handle"):
        dcn_forward_numpy(x, wo, bo, w, b, s, (1, 1), state=st)
    st.close()
