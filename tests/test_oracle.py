"""CPU: pin the oracles (NumPy float64 + C fp32) against the golden fixtures.

The fixtures (tests/golden/make_golden.py) are a literal torch restatement of
deform_conv.py:56-81 run in fp32 like the reference; the float64 twins check the
NumPy oracle beyond fp32 noise. No reference golden vectors exist,
so this is the strongest pin available without Jittor (parity unpinned w.r.t.
the Jittor runtime itself).
"""
import numpy as np
import pytest

import dcn_oracle as O
import ref_lib as R
from conftest import assert_close, assert_close_reduction, golden_names, load_golden

GRAD_KEYS = [("x", "grad_x", "elem"), ("weight", "grad_weight", "red"),
             ("offset_conv.weight", "grad_offset_weight", "red"),
             ("offset_conv.bias", "grad_offset_bias", "red"), ("offset", "grad_offset", "elem")]


def _check_all(out, off, grads, d, prefix, what):
    assert_close(out, d[prefix + "out"], what=f"{what} out")
    assert_close(off, d[prefix + "off"], what=f"{what} offset")
    for k, gk, kind in GRAD_KEYS:
        if kind == "elem":
            assert_close(grads[k], d[prefix + gk], what=f"{what} ∂{k}")
        else:
            assert_close_reduction(grads[k], d[prefix + gk], what=f"{what} ∂{k}")
    if d["b"] is not None:
        assert_close_reduction(grads["bias"], d[prefix + "grad_bias"], what=f"{what} ∂bias")


@pytest.mark.parametrize("name", golden_names())
def test_numpy_oracle_vs_golden_f32(name):
    d = load_golden(name)
    out, off, cache = O.forward(d["x"], d["w_off"], d["b_off"], d["w"], d["b"], d["stride"],
                                d["padding"])
    g = O.backward(cache, d["grad_out"])
    _check_all(out, off, g, d, "f32_", name)


@pytest.mark.parametrize("name", [n for n in golden_names() if "f64_out" in load_golden(n)])
def test_numpy_oracle_vs_golden_f64(name):
    d = load_golden(name)
    out, off, cache = O.forward(d["x"], d["w_off"], d["b_off"], d["w"], d["b"], d["stride"],
                                d["padding"])
    g = O.backward(cache, d["grad_out"])
    # only fp32 coordinate rounding separates the two (random offsets, no knife edge)
    assert_close(out, d["f64_out"], atol=2e-5, rtol=2e-5, what="out")
    for k, gk, _ in GRAD_KEYS:
        assert_close(g[k], d["f64_" + gk], atol=3e-4, rtol=3e-5, what=f"∂{k}")


@pytest.mark.parametrize("name", golden_names())
def test_c_oracle_vs_golden(name):
    d = load_golden(name)
    desc = R.make_desc(d["x"].shape, d["w"].shape, d["stride"], d["padding"],
                       has_bias=d["b"] is not None)
    out, off = R.forward(desc, d["x"], d["w_off"], d["b_off"], d["w"], d["b"])
    g = R.backward(desc, d["x"], off, d["w_off"], d["w"], d["grad_out"])
    _check_all(out, off, g, d, "f32_", name)


def test_zero_offsets_are_a_transposed_linear_map():
    """Q1/Q3: with zero offsets and a square stride-1 map every tap samples input
    (row=w, col=h): out[b,o,h,w] = bias + Σ_c (Σ_n W[o][n][c]) x[b,c,w,h]."""
    rng = np.random.default_rng(7)
    B, C, O_, H = 2, 3, 4, 9
    x = rng.standard_normal((B, C, H, H)).astype(np.float32)
    w = rng.standard_normal((O_, C, 3, 3)).astype(np.float32)
    b = rng.standard_normal(O_).astype(np.float32)
    wo = np.zeros((18, C, 3, 3), np.float32)
    bo = np.zeros(18, np.float32)
    out, _, _ = O.forward(x, wo, bo, w, b, (1, 1), (1, 1))
    Wsum = O.weight_matrix(w).sum(axis=1)  # [O, C]
    expect = np.einsum("oc,bcwh->bohw", Wsum, x.astype(np.float64)) + b[None, :, None, None]
    # knife-edge floors (Q6) make a few taps interpolate at fraction 1.0 from the
    # row below: value identical, so the map is exact up to fp rounding
    np.testing.assert_allclose(out, expect, rtol=1e-5, atol=1e-5)


def test_weight_is_read_as_o_n_c():
    """Q5: perturbing flat weight index o*N*C + n*C + c changes the result exactly
    like column k = n*C + c of the sampled matrix."""
    rng = np.random.default_rng(3)
    x = rng.standard_normal((1, 2, 6, 6)).astype(np.float32)
    wo = (rng.standard_normal((18, 2, 3, 3)) * 0.3).astype(np.float32)
    bo = rng.uniform(-1, 1, 18).astype(np.float32)
    w = np.zeros((1, 2, 3, 3), np.float32)
    n, c = 4, 1
    w.reshape(-1)[n * 2 + c] = 1.0
    out, off, _ = O.forward(x, wo, bo, w, None, (1, 1), (1, 1))
    col = O.im2col(x, off, 3, 3)
    np.testing.assert_allclose(out[0, 0].reshape(-1), col[0, n * 2 + c], rtol=1e-12, atol=1e-12)


@pytest.mark.parametrize("dil,G", [((2, 2), 1), ((1, 1), 2), ((2, 2), 4)])
def test_extension_numpy_vs_c(dil, G):
    """Extensions (dilation, deform_groups; config 5): no reference oracle exists
    ("parity unpinned"), so the two restatements are checked against each other,
    and against the reference semantics when dil=1, G=1 (the cases above)."""
    rng = np.random.default_rng(11)
    B, C, O_, H, W = 2, 8, 5, 14, 13
    s, p = (2, 2), (1, 1)
    N = 9
    x = rng.standard_normal((B, C, H, W)).astype(np.float32)
    wo = (rng.standard_normal((2 * N * G, C, 3, 3)) * 0.4 / np.sqrt(C * 9)).astype(np.float32)
    bo = rng.uniform(-1, 1, 2 * N * G).astype(np.float32)
    w = (rng.standard_normal((O_, C, 3, 3)) * np.sqrt(2 / (C * 9))).astype(np.float32)
    b = rng.standard_normal(O_).astype(np.float32)
    out, off, cache = O.forward(x, wo, bo, w, b, s, p, dil, G)
    Ho, Wo = off.shape[2:]
    gout = rng.standard_normal((B, O_, Ho, Wo)).astype(np.float32)
    g = O.backward(cache, gout)
    desc = R.make_desc(x.shape, w.shape, s, p, dil, G, True)
    out_c, off_c = R.forward(desc, x, wo, bo, w, b)
    g_c = R.backward(desc, x, off_c, wo, w, gout)
    assert_close(out_c, out, what="out")
    assert_close(off_c, off, what="offset")
    assert_close(g_c["x"], g["x"], what="∂x")
    assert_close(g_c["offset"], g["offset"], what="∂offset")
    assert_close_reduction(g_c["weight"], g["weight"], what="∂W")
    assert_close_reduction(g_c["offset_conv.weight"], g["offset_conv.weight"], what="∂W_off")
    assert_close_reduction(g_c["offset_conv.bias"], g["offset_conv.bias"], what="∂b_off")


def test_out_size_matches_reference_formula():
    # deform_conv.py:34-35 (dilation 1) for the EDNet layers (train.py:311-320)
    for H in (128, 64, 32, 16):
        assert O.out_size(H, H, 3, 3, 2, 2, 1, 1) == (H // 2, H // 2)
    assert O.out_size(14, 14, 3, 3, 2, 2, 1, 1, 2, 2) == (6, 6)  # config 5
