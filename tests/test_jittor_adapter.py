"""The Jittor backend of jittor-dcn_amd/deform_conv.py (`DeformConv2d` as a jt.Module whose
execute is a jt.Function), driven through a stand-in of Jittor's Function protocol
(tests/jittor_standin.py) because Jittor is not installable here.

What this pins is the adapter's contract with Jittor autodiff as the reference's caller
uses it (train.py:329-332 builds the model, :414 optimizer.backward reaches `grad`):
  * the constructor keeps the reference's surface (deform_conv.py:7-28): tuples, N, a
    zero-initialised offset conv [2N, C, kh, kw], weight [O, C, kh, kw], bias or None;
  * `grad` returns one entry per `execute` input, in order, None for the non-Var ones
    (stride / padding, and the bias when bias=False), and the Var grads equal the oracle's.
CPU: libdcn's host calls are replaced by the NumPy oracle (the adapter's plumbing only).
GPU: the real libdcn path. Parity with Jittor itself stays unpinned.
"""
import importlib.util
import os

import numpy as np
import pytest

import dcn_oracle as O
import jittor_standin
from conftest import PKG, assert_close, assert_close_reduction


@pytest.fixture()
def jdc():
    jt = jittor_standin.install()
    try:
        spec = importlib.util.spec_from_file_location("deform_conv_jt",
                                                      os.path.join(PKG, "deform_conv.py"))
        mod = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(mod)
        assert mod.HAVE_JITTOR
        yield jt, mod
    finally:
        jittor_standin.uninstall()


def _oracle_fwd(x, w_off, b_off, w, b, stride, padding, return_ctx=False, **kw):
    out, off, _ = O.forward(x, w_off, b_off, w, b, stride, padding)
    res = out.astype(np.float32), off.astype(np.float32)
    return res + (None,) if return_ctx else res


def _oracle_bwd(x, off, w_off, w, has_bias, grad_out, stride, padding, **kw):
    b = np.zeros(w.shape[0], np.float32)
    _, _, cache = O.forward(x, w_off, np.zeros(w_off.shape[0], np.float32), w, b, stride,
                            padding, offsets=off)
    g = O.backward(cache, grad_out)
    if not has_bias:
        g.pop("bias", None)
    return g


def _drive(jt, mod, bias, seed=3):
    rng = np.random.default_rng(seed)
    m = mod.DeformConv2d(6, 5, 3, 2, 1, bias=bias)
    # reference surface (deform_conv.py:9-28)
    assert m.kernel_size == (3, 3) and m.stride == (2, 2) and m.padding == (1, 1) and m.N == 9
    assert m.offset_conv.weight.shape == (18, 6, 3, 3) and not m.offset_conv.weight.numpy().any()
    assert m.offset_conv.bias.shape == (18,) and not m.offset_conv.bias.numpy().any()
    assert m.weight.shape == (5, 6, 3, 3)
    assert (m.bias is None) == (not bias)
    # non-zero offsets so the sampling path is exercised
    m.offset_conv.weight = jt.array(rng.standard_normal((18, 6, 3, 3)) * 0.3)
    m.offset_conv.bias = jt.array(rng.uniform(-1, 1, 18))
    if bias:
        m.bias = jt.array(rng.standard_normal(5) * 0.1)
    x = rng.standard_normal((2, 6, 11, 9)).astype(np.float32)
    out = m(jt.array(x))
    f = jt.Function.last
    gout = rng.standard_normal(out.shape).astype(np.float32)
    grads = f.backward(jt.array(gout))
    w_off, b_off = m.offset_conv.weight.numpy(), m.offset_conv.bias.numpy()
    b = m.bias.numpy() if bias else None
    ro, _, cache = O.forward(x, w_off, b_off, m.weight.numpy(), b, (2, 2), (1, 1))
    rg = O.backward(cache, gout)
    return out, grads, ro, rg


@pytest.mark.parametrize("bias", [True, False])
def test_jittor_adapter_grad_contract_cpu(jdc, monkeypatch, bias):
    jt, mod = jdc
    monkeypatch.setattr(mod, "dcn_forward_numpy", _oracle_fwd)
    monkeypatch.setattr(mod, "dcn_backward_numpy", _oracle_bwd)
    out, grads, ro, rg = _drive(jt, mod, bias)
    np.testing.assert_allclose(out.numpy(), ro, rtol=1e-6, atol=1e-6)
    # Var inputs in execute order: x, offset_conv.weight, offset_conv.bias, weight, (bias)
    names = ["x", "offset_conv.weight", "offset_conv.bias", "weight"] + (["bias"] if bias else [])
    assert len(grads) == len(names)
    for n, gv in zip(names, grads):
        np.testing.assert_allclose(gv.numpy(), rg[n], rtol=1e-5, atol=1e-5, err_msg=n)


@pytest.mark.gpu
@pytest.mark.parametrize("bias", [True, False])
def test_jittor_adapter_on_libdcn(jdc, bias):
    jt, mod = jdc
    out, grads, ro, rg = _drive(jt, mod, bias, seed=4)
    assert_close(out.numpy(), ro, what="jt adapter out")
    names = ["x", "offset_conv.weight", "offset_conv.bias", "weight"] + (["bias"] if bias else [])
    assert len(grads) == len(names)
    assert_close(grads[0].numpy(), rg["x"], what="jt adapter ∂x")
    for n, gv in zip(names[1:], grads[1:]):
        assert_close_reduction(gv.numpy(), rg[n], what=f"jt adapter ∂{n}")


def test_jittor_adapter_empty_batch(jdc):
    """An empty batch through the jt.Function: execute unpacks the forward's
    (out, off, ctx) and grad returns zero parameter grads, with no launch."""
    jt, mod = jdc
    m = mod.DeformConv2d(4, 6, 3, 1, 1)
    out = m(jt.array(np.zeros((0, 4, 8, 8), np.float32)))
    assert out.shape == (0, 6, 8, 8)
    grads = jt.Function.last.backward(jt.array(np.zeros((0, 6, 8, 8), np.float32)))
    assert grads[0].shape == (0, 4, 8, 8)
    for gv in grads[1:5]:
        assert not gv.numpy().any()
