"""GPU parity of the bf16 fused forward (csrc/dcn_fused_bf16.hip): the
bilinear gather of deform_conv.py:47-54 fed from an LDS window of the channels-last x straight
into the B operand of bf16 MFMAs computing :76-80, the columns written only for a backward
that reuses them (DCN_FWD_FUSED) or never (DCN_FWD_FUSED_NOCOL).

* against the unfused schedule (K1 + hipBLASLt + bias, DCN_FWD_UNFUSED) on the same handle:
  out within one bf16 rounding of a different fp32 summation order; the columns the fused
  kernel stores bit for bit K1's, checked through the backward, whose ∂W GEMM reads them
  (DCN_BWD_COL_IN_WS): every gradient identical;
* DCN_FWD_FUSED_NOCOL (no column matrix anywhere in the step): out bit for bit the storing
  kernel's; its backward computes ∂W with the columns recomputed inside the MFMA kernel
  (dw_fused_bf16): ∂W within one bf16 rounding of the GEMM schedule's (another fp32 summation
  order) and against the oracle, every other gradient bit for bit;
* against the oracle (the bf16 tolerance of test_gpu_bf16);
* many samples outside the tile's LDS window (offset scale 3-8 px): the per-tile overflow
  area and, past its 48 entries, the in-line global corner reads;
* config 4 at full size: forward twice in one process, bit for bit.
"""
import numpy as np
import pytest

import dcn_oracle as O
import dcn_runtime as rt
from test_gpu_bf16 import _case, _device, assert_bf16_close

pytestmark = pytest.mark.gpu

CASES = [
    dict(seed=901, B=2, C=256, O_=256, H=28, W=28),                 # config 4 geometry
    dict(seed=902, B=2, C=64, O_=256, H=20, W=17, off_scale=2.0),   # ragged tiles (7x16)
    dict(seed=903, B=3, C=128, O_=512, H=24, W=24, s=(2, 2)),       # stride 2, 2 O tiles
    dict(seed=904, B=1, C=64, O_=256, H=9, W=40, k=(3, 2), p=(1, 0)),  # 6 taps, 3 tile cols
    dict(seed=905, B=2, C=192, O_=256, H=15, W=30, off_scale=3.0),  # overflow area in use
    dict(seed=906, B=2, C=64, O_=256, H=16, W=16, off_scale=8.0),   # past the overflow area
    dict(seed=907, B=2, C=64, O_=256, H=11, W=13, k=(1, 1), p=(0, 0)),  # 1 tap
]


def _run(h, c, path, pad=None):
    bits, v, s = c
    h.set_fwd_path(path)
    try:
        return _device(h, bits, s, pad=pad or (1, 1))
    finally:
        h.set_fwd_path(rt.DCN_FWD_AUTO)


def _pad(case):
    return case.get("p", (1, 1))


def _near(a, r, what):
    """One bf16 rounding of two fp32 sums that differ only in summation order."""
    d = np.abs(a.astype(np.float64) - r)
    rms = float(np.sqrt(np.mean(r.astype(np.float64) ** 2)))
    lim = 2.0 ** -7 * np.abs(r) + 2.0 ** -14 * rms
    assert np.all(d <= lim), f"{what}: {int((d > lim).sum())} elements past one bf16 ulp"


@pytest.mark.parametrize("case", CASES)
def test_fused_bf16_vs_unfused_and_oracle(gpu_handle, case):
    c = _case(**case)
    pad = _pad(case)
    out_f, off_f, g_f = _run(gpu_handle, c, rt.DCN_FWD_FUSED, pad)
    out_u, off_u, g_u = _run(gpu_handle, c, rt.DCN_FWD_UNFUSED, pad)
    np.testing.assert_array_equal(off_f, off_u)
    _near(out_f, out_u, f"fused vs unfused out {case}")
    # the stored columns are K1's bit for bit -> the whole backward is bitwise equal
    for k in g_u:
        np.testing.assert_array_equal(g_f[k], g_u[k], err_msg=f"∂{k} (columns differ) {case}")
    _, v, s = c
    ro, _, _ = O.forward(v["x"], v["w_off"], v["b_off"], v["w"], v["b"], s, pad, offsets=off_f)
    assert_bf16_close(out_f, ro, f"fused out vs oracle {case}")


@pytest.mark.parametrize("case", CASES)
def test_fused_bf16_nocol(gpu_handle, case):
    c = _case(**case)
    pad = _pad(case)
    out_f, _, _ = _run(gpu_handle, c, rt.DCN_FWD_FUSED, pad)
    out_n, off_n, g_n = _run(gpu_handle, c, rt.DCN_FWD_FUSED_NOCOL, pad)
    _, _, g_u = _run(gpu_handle, c, rt.DCN_FWD_UNFUSED, pad)
    np.testing.assert_array_equal(out_n.view(np.uint32), out_f.view(np.uint32))
    for k in g_u:
        if k == "weight":  # recomputed columns, another fp32 summation order
            _near(g_n[k], g_u[k], f"nocol ∂W vs GEMM {case}")
        else:
            np.testing.assert_array_equal(g_n[k], g_u[k], err_msg=f"nocol ∂{k}")
    _, v, s = c
    _, _, cache = O.forward(v["x"], v["w_off"], v["b_off"], v["w"], v["b"], s, pad,
                            offsets=off_n)
    rg = O.backward(cache, v["grad_out"])
    assert_bf16_close(g_n["weight"], rg["weight"], f"nocol ∂W vs oracle {case}")


def test_fused_bf16_config4_full_size_bitwise(gpu_handle):
    """BASELINE config 4 per GPU (B=64, C=O=256, 28x28): the fused forward twice in one
    process, bit for bit, and against the unfused schedule within one bf16 rounding."""
    c = _case(12, B=64, C=256, O_=256, H=28, W=28, off_scale=1.5)
    r1 = _run(gpu_handle, c, rt.DCN_FWD_FUSED)
    r2 = _run(gpu_handle, c, rt.DCN_FWD_FUSED)
    np.testing.assert_array_equal(r1[0].view(np.uint32), r2[0].view(np.uint32), err_msg="out")
    for k in r1[2]:
        np.testing.assert_array_equal(r1[2][k].view(np.uint32), r2[2][k].view(np.uint32),
                                      err_msg=k)
    ru = _run(gpu_handle, c, rt.DCN_FWD_UNFUSED)
    _near(r1[0], ru[0], "config 4 fused vs unfused out")
    for k in ru[2]:
        np.testing.assert_array_equal(r1[2][k], ru[2][k], err_msg=f"config 4 ∂{k}")


def test_fused_bf16_nocol_config4_full_size(gpu_handle):
    """BASELINE config 4 per GPU with no column matrix (fused forward, recomputed ∂W): twice
    in one process bit for bit, and against the column schedule (∂W within one bf16
    rounding, every other tensor bit for bit)."""
    c = _case(13, B=64, C=256, O_=256, H=28, W=28, off_scale=1.5)
    r1 = _run(gpu_handle, c, rt.DCN_FWD_FUSED_NOCOL)
    r2 = _run(gpu_handle, c, rt.DCN_FWD_FUSED_NOCOL)
    np.testing.assert_array_equal(r1[0].view(np.uint32), r2[0].view(np.uint32), err_msg="out")
    for k in r1[2]:
        np.testing.assert_array_equal(r1[2][k].view(np.uint32), r2[2][k].view(np.uint32),
                                      err_msg=k)
    ru = _run(gpu_handle, c, rt.DCN_FWD_UNFUSED)
    _near(r1[0], ru[0], "config 4 nocol vs unfused out")
    for k in ru[2]:
        if k == "weight":
            _near(r1[2][k], ru[2][k], "config 4 nocol ∂W")
        else:
            np.testing.assert_array_equal(r1[2][k], ru[2][k], err_msg=f"config 4 nocol ∂{k}")
