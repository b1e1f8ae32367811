"""GPU parity of the fused forward (dcn_fused.hip): the bilinear im2col
gathered straight into the f32 MFMA GEMM's LDS tiles, bias in the epilogue.

* against the oracle (tolerance of the north star, conftest.assert_close);
* against the unfused schedule (K1 + vendor GEMM + bias, DCN_FWD_UNFUSED) on the same
  handle: the output to fp32 rounding of a different summation order, and the columns the
  fused kernel leaves in the workspace bit for bit — checked through the backward, whose
  ∂W GEMM reads them (DCN_BWD_COL_IN_WS): every gradient must then be identical.
"""
import numpy as np
import pytest

import dcn_runtime as rt
from conftest import assert_close
from test_gpu_parity import _check, _device_fwd_bwd, _oracle, _rand_case

pytestmark = pytest.mark.gpu

CASES = [
    dict(seed=81, B=2, C=32, O_=128, H=13, W=13),                 # HW 169: ragged last tile
    dict(seed=82, B=2, C=64, O_=256, H=20, W=18, off_scale=2.0),   # OT 256, HW not /64
    dict(seed=83, B=1, C=96, O_=384, H=9, W=11, bias=False),       # OT 128 x 3 O tiles
    dict(seed=84, B=3, C=32, O_=128, H=24, W=24, s=(2, 2)),        # stride 2 (EDNet-like)
    dict(seed=85, B=2, C=64, O_=128, H=16, W=16, off_scale=8.0),   # many samples off-image
    dict(seed=86, B=2, C=32, O_=128, H=12, W=14, k=(3, 2), p=(1, 0)),  # 6 taps
]


def _run(h, c, path):
    h.set_fwd_path(path)
    try:
        return _device_fwd_bwd(h, c)
    finally:
        h.set_fwd_path(rt.DCN_FWD_AUTO)


@pytest.mark.parametrize("case", CASES)
def test_fused_forward_vs_oracle(gpu_handle, case):
    c = _rand_case(**case)
    out, off, g = _run(gpu_handle, c, rt.DCN_FWD_FUSED)
    ro, roff, rg = _oracle(c, off)
    _check(out, off, g, ro, roff, rg, c["b"] is not None, f"fused {case}")


@pytest.mark.parametrize("case", CASES[:4])
def test_fused_forward_vs_unfused(gpu_handle, case):
    c = _rand_case(**case)
    out_f, off_f, g_f = _run(gpu_handle, c, rt.DCN_FWD_FUSED)
    out_u, off_u, g_u = _run(gpu_handle, c, rt.DCN_FWD_UNFUSED)
    np.testing.assert_array_equal(off_f, off_u)
    # same products, different summation order: a few fp32 ulps of the row magnitude
    scale = np.abs(out_u).max()
    assert np.abs(out_f - out_u).max() <= 1e-5 * scale, "fused vs unfused out"
    # columns in the workspace bit-identical -> the whole backward is bitwise equal
    for k in g_u:
        np.testing.assert_array_equal(g_f[k], g_u[k], err_msg=f"∂{k} (columns differ)")


@pytest.mark.parametrize("nwg", [1, 3, 7])
def test_fused_few_workgroups_walk_tiles(gpu_handle, nwg):
    """A persistent workgroup walks many 128-px tiles, some straddling two images, and a
    ragged last block (B·Ho·Wo = 3·13·15 = 585 pixels = 18.3 blocks)."""
    c = _rand_case(88 + nwg, B=3, C=64, O_=256, H=13, W=15, off_scale=2.0)
    rt.check(gpu_handle.lib.dcn_debug_fused_workgroups(nwg))
    try:
        out_f, off_f, g_f = _run(gpu_handle, c, rt.DCN_FWD_FUSED)
    finally:
        rt.check(gpu_handle.lib.dcn_debug_fused_workgroups(0))
    out_u, off_u, g_u = _run(gpu_handle, c, rt.DCN_FWD_UNFUSED)
    scale = np.abs(out_u).max()
    assert np.abs(out_f - out_u).max() <= 1e-5 * scale, f"fused nwg={nwg} vs unfused out"
    for k in g_u:
        np.testing.assert_array_equal(g_f[k], g_u[k], err_msg=f"nwg={nwg} ∂{k}")
    ro, roff, rg = _oracle(c, off_f)
    _check(out_f, off_f, g_f, ro, roff, rg, True, f"fused nwg={nwg}")


def test_fused_path_rejects_unknown_mode(gpu_handle):
    with pytest.raises(RuntimeError):
        gpu_handle.set_fwd_path(7)
    with pytest.raises(RuntimeError):
        rt.check(gpu_handle.lib.dcn_debug_fused_workgroups(-1))


def test_fused_config3_tile_vs_oracle(gpu_handle):
    """Config-3 channel counts (C = O = 256) on a small image batch: OT = 256 tiles."""
    c = _rand_case(87, B=2, C=256, O_=256, H=15, W=17)
    out, off, g = _run(gpu_handle, c, rt.DCN_FWD_FUSED)
    ro, roff, rg = _oracle(c, off)
    assert_close(out, ro, what="fused C=O=256 out")
