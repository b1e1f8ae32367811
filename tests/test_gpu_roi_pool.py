"""GPU parity: libdcn's deformable RoI pooling (deform_conv.py:85-241)
against the oracle (pinned to a literal torch restatement in test_roi_pool_oracle.py).

Tolerance: |Δ| <= 1e-4 + 1e-4·|ref| for the pooled values and ∂features (the north star's
fp32 bar); ∂offsets are channel reductions: max|Δ|/max|ref| <= 1e-4.
"""
import numpy as np
import pytest

import dcn_oracle as O
from conftest import assert_close, assert_close_reduction
from deform_conv import (DeformPSRoIPoolNumpy, DeformRoIPoolNumpy, roi_pool_backward_numpy,
                         roi_pool_forward_numpy)
from test_roi_pool_oracle import CASES, roi_case

pytestmark = pytest.mark.gpu


def _run(case, feat, rois, offsets, h):
    c = dict(case)
    ps = c.pop("kind") == "ps"
    P = c["output_size"][0] * c["output_size"][1]
    offs = offsets.reshape(len(rois), 2 * P) if ps else offsets
    kw = dict(ps=ps, part_size=c.get("part_size"), trans_std=c.get("trans_std", 0.1),
              no_trans=c.get("no_trans", False))
    out = roi_pool_forward_numpy(feat, rois, offs, c["output_size"], c["spatial_scale"],
                                 handle=h, **kw)
    ref = O.roi_pool_forward(feat, rois, offsets, c["output_size"], c["spatial_scale"], **kw)
    g = np.random.default_rng(11).standard_normal(out.shape).astype(np.float32)
    gf, go = roi_pool_backward_numpy(feat, rois, offs, g, c["output_size"], c["spatial_scale"],
                                     handle=h, **kw)
    rgf, rgo = O.roi_pool_backward(feat, rois, offsets, g, c["output_size"], c["spatial_scale"],
                                   **kw)
    return out, ref, gf, rgf, go.reshape(len(rois), P, 2), rgo


@pytest.mark.parametrize("case", CASES, ids=lambda c: "-".join(f"{k}={v}" for k, v in c.items()))
def test_roi_pool_vs_oracle(gpu_handle, case):
    P = case["output_size"][0] * case["output_size"][1]
    feat, rois, offsets = roi_case(21, P=P)
    out, ref, gf, rgf, go, rgo = _run(case, feat, rois, offsets, gpu_handle)
    assert_close(out, ref, what="pooled")
    assert_close(gf, rgf, what="∂features")
    if case.get("no_trans"):
        assert not go.any()
    else:
        assert_close_reduction(go, rgo, what="∂offsets")


def test_roi_pool_large_shared_pixels(gpu_handle):
    """Many RoIs over one feature map (pixels shared by RoIs: the atomic ∂features path),
    C = 256 (one channel per lane), RoIs partly outside the image."""
    rng = np.random.default_rng(5)
    B, C, H, W, R = 2, 256, 32, 40, 300
    feat = rng.standard_normal((B, C, H, W)).astype(np.float32)
    xy = rng.uniform(-4, 36, (R, 2))
    rois = np.concatenate([rng.integers(0, B, (R, 1)), xy, xy + rng.uniform(1, 12, (R, 2))],
                          axis=1).astype(np.float32)
    offsets = (rng.standard_normal((R, 1, 2)) * 0.2).astype(np.float32)
    for case in (dict(kind="roi", output_size=(1, 1), spatial_scale=0.5),
                 dict(kind="ps", output_size=(1, 1), spatial_scale=0.5, trans_std=0.1)):
        out, ref, gf, rgf, go, rgo = _run(case, feat, rois, offsets, gpu_handle)
        assert_close(out, ref, what=f"{case['kind']} pooled")
        assert_close(gf, rgf, what=f"{case['kind']} ∂features")
        assert_close_reduction(go, rgo, what=f"{case['kind']} ∂offsets")


def test_roi_pool_modules_match_reference_surface(gpu_handle):
    """Module surface of deform_conv.py:85-91 / :162-172: output [R, C, 1, 1] for a 1x1
    output; for ph*pw != 1 the reference's final reshape fails, and so does ours."""
    feat, rois, offsets = roi_case(3, C=8, P=1)
    m = DeformRoIPoolNumpy(1, spatial_scale=1.0)
    out = m(feat, rois, offsets)
    assert out.shape == (len(rois), 8, 1, 1)
    gf, go = m.backward(np.ones_like(out))
    assert gf.shape == feat.shape and go.shape == offsets.shape
    ps = DeformPSRoIPoolNumpy((1, 1), trans_std=0.1)
    assert ps(feat, rois, offsets.reshape(len(rois), 2)).shape == (len(rois), 8, 1, 1)
    _, rois2, off2 = roi_case(3, C=8, P=4)
    with pytest.raises(ValueError):
        DeformRoIPoolNumpy((2, 2))(feat, rois2, off2)


def test_roi_pool_rejects_bad_batch_index(gpu_handle):
    feat, rois, offsets = roi_case(4, B=2, P=1)
    rois[1, 0] = 2.0
    with pytest.raises(RuntimeError, match="batch index"):
        roi_pool_forward_numpy(feat, rois, offsets, (1, 1), handle=gpu_handle)


@pytest.mark.parametrize("B,C,H,W,R", [(1, 3, 7, 5, 9), (3, 70, 16, 13, 17), (2, 300, 10, 12, 6),
                                       (4, 64, 21, 9, 33), (1, 129, 5, 30, 8)])
@pytest.mark.parametrize("kind,out_size", [("roi", (1, 1)), ("ps", (2, 2))])
def test_roi_pool_shapes_vs_oracle(gpu_handle, B, C, H, W, R, kind, out_size):
    """Feature-map and channel shapes beside the fixed cases: C below, between and above the
    64-lane block (3, 70, 129, 300), tall/wide maps, more RoIs than the batch."""
    P = out_size[0] * out_size[1]
    if kind == "ps" and C < P:
        pytest.skip("PS pooling needs C >= ph·pw channels (C // (ph·pw) output channels)")
    feat, rois, offsets = roi_case(40 + C, B=B, C=C, H=H, W=W, R=R, P=P)
    case = dict(kind=kind, output_size=out_size, spatial_scale=0.75)
    out, ref, gf, rgf, go, rgo = _run(case, feat, rois, offsets, gpu_handle)
    assert_close(out, ref, what="pooled")
    assert_close(gf, rgf, what="∂features")
    assert_close_reduction(go, rgo, what="∂offsets")
