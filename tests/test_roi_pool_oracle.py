"""CPU: the deformable RoI pooling oracle (oracle/dcn_oracle.py, roi_*) against a literal
op-for-op torch restatement of deform_conv.py:85-159 (DeformRoIPool) and :162-241
(DeformPSRoIPool), forward and autograd.

The restatement below follows the reference line by line (jt.* -> torch.*), in fp32 like
the reference. The reference's own tests never exercise these modules (SURVEY §8(f) f4:
unused by train.py/test.py), and Jittor is not installable here, so this pins the oracle
to the reference's algorithm, not to the Jittor runtime: parity unpinned w.r.t. Jittor.
Both stop at the reference's `.sum(dim=2)` (the value before its reshape, which only
succeeds for ph*pw == 1).
"""
import numpy as np
import pytest
import torch

import dcn_oracle as O


def torch_roi_pool(features, rois, offsets, output_size, spatial_scale=1.0):
    """deform_conv.py:92-158 up to the reshape, fp32."""
    B, C, H, W = features.shape
    num_rois = rois.shape[0]
    pooled_h, pooled_w = output_size
    batch_indices = rois[:, 0].long()
    roi_coords = rois[:, 1:5] * spatial_scale
    x1, y1, x2, y2 = roi_coords[:, 0], roi_coords[:, 1], roi_coords[:, 2], roi_coords[:, 3]
    roi_w = torch.clamp(x2 - x1, min=1e-6)
    roi_h = torch.clamp(y2 - y1, min=1e-6)
    ph = torch.arange(pooled_h, dtype=torch.float32)
    pw = torch.arange(pooled_w, dtype=torch.float32)
    ph_grid, pw_grid = torch.meshgrid(ph, pw, indexing="ij")
    ph_grid = ph_grid.reshape(-1)
    pw_grid = pw_grid.reshape(-1)
    bin_w = roi_w[:, None] / pooled_w
    bin_h = roi_h[:, None] / pooled_h
    bin_cx = x1[:, None] + (pw_grid + 0.5) * bin_w
    bin_cy = y1[:, None] + (ph_grid + 0.5) * bin_h
    idx = (ph_grid * pooled_w + pw_grid).long()
    offset_x = offsets[:, idx, 0] * roi_w[:, None]
    offset_y = offsets[:, idx, 1] * roi_h[:, None]
    cx = bin_cx + offset_x
    cy = bin_cy + offset_y
    x0 = torch.floor(cx).long()
    x1 = x0 + 1
    y0 = torch.floor(cy).long()
    y1 = y0 + 1
    x0 = torch.clamp(x0, 0, W - 1)
    x1 = torch.clamp(x1, 0, W - 1)
    y0 = torch.clamp(y0, 0, H - 1)
    y1 = torch.clamp(y1, 0, H - 1)
    dx = cx - x0.float()
    dy = cy - y0.float()
    w00 = (1 - dx) * (1 - dy)
    w01 = (1 - dx) * dy
    w10 = dx * (1 - dy)
    w11 = dx * dy
    P = pooled_h * pooled_w
    batch_idx = batch_indices[:, None].repeat(1, P)
    out = 0
    for (yy, xx, ww) in ((y0, x0, w00), (y1, x0, w01), (y0, x1, w10), (y1, x1, w11)):
        feats = features[batch_idx.reshape(-1), :, yy.reshape(-1), xx.reshape(-1)]
        feats = feats.reshape(num_rois, P, C).permute(0, 2, 1)
        out = out + (feats * ww[:, None, :]).sum(dim=2)
    return out


def torch_psroi_pool(features, rois, offsets, output_size, spatial_scale=1.0, no_trans=False,
                     part_size=None, trans_std=0.1):
    """deform_conv.py:174-240 up to the reshape, fp32."""
    B, C, H, W = features.shape
    num_rois = rois.shape[0]
    pooled_h, pooled_w = output_size
    part_h, part_w = part_size if part_size else output_size
    C_out = C // (pooled_h * pooled_w)
    batch_indices = rois[:, 0].long()
    roi_coords = rois[:, 1:5] * spatial_scale
    x1, y1, x2, y2 = roi_coords[:, 0], roi_coords[:, 1], roi_coords[:, 2], roi_coords[:, 3]
    roi_w = torch.clamp(x2 - x1, min=1e-6)
    roi_h = torch.clamp(y2 - y1, min=1e-6)
    ph = torch.arange(pooled_h, dtype=torch.float32)
    pw = torch.arange(pooled_w, dtype=torch.float32)
    ph_grid, pw_grid = torch.meshgrid(ph, pw, indexing="ij")
    ph_flat = ph_grid.reshape(-1)
    pw_flat = pw_grid.reshape(-1)
    part_idx = ph_flat * pooled_w + pw_flat
    bin_w = roi_w[:, None] / part_w
    bin_h = roi_h[:, None] / part_h
    bin_cx = x1[:, None] + (pw_flat + 0.5) * bin_w
    bin_cy = y1[:, None] + (ph_flat + 0.5) * bin_h
    if not no_trans:
        trans_x = offsets[:, (part_idx * 2).long()] * roi_w[:, None] * trans_std
        trans_y = offsets[:, (part_idx * 2 + 1).long()] * roi_h[:, None] * trans_std
        cx = bin_cx + trans_x
        cy = bin_cy + trans_y
    else:
        cx = bin_cx
        cy = bin_cy
    x0 = torch.floor(cx).long()
    x1 = x0 + 1
    y0 = torch.floor(cy).long()
    y1 = y0 + 1
    x0 = torch.clamp(x0, 0, W - 1)
    x1 = torch.clamp(x1, 0, W - 1)
    y0 = torch.clamp(y0, 0, H - 1)
    y1 = torch.clamp(y1, 0, H - 1)
    dx = cx - x0.float()
    dy = cy - y0.float()
    w00 = (1 - dx) * (1 - dy)
    w01 = (1 - dx) * dy
    w10 = dx * (1 - dy)
    w11 = dx * dy
    P = pooled_h * pooled_w
    c_out = torch.arange(C_out)[:, None]
    channel_idx = (c_out * P + part_idx.long()).repeat(num_rois, 1, 1)
    batch_idx = batch_indices[:, None, None].repeat(1, C_out, P)
    y0_, x0_ = y0[:, None, :].repeat(1, C_out, 1), x0[:, None, :].repeat(1, C_out, 1)
    y1_, x1_ = y1[:, None, :].repeat(1, C_out, 1), x1[:, None, :].repeat(1, C_out, 1)
    val00 = features[batch_idx, channel_idx, y0_, x0_] * w00[:, None, :]
    val01 = features[batch_idx, channel_idx, y1_, x0_] * w01[:, None, :]
    val10 = features[batch_idx, channel_idx, y0_, x1_] * w10[:, None, :]
    val11 = features[batch_idx, channel_idx, y1_, x1_] * w11[:, None, :]
    return (val00 + val01 + val10 + val11).sum(dim=2)


def roi_case(seed, B=2, C=12, H=9, W=11, R=5, P=1):
    rng = np.random.default_rng(seed)
    feat = rng.standard_normal((B, C, H, W)).astype(np.float32)
    b = rng.integers(0, B, R)
    xy = rng.uniform(-3, 12, (R, 2))
    wh = rng.uniform(0.5, 8, (R, 2))
    rois = np.concatenate([b[:, None], xy, xy + wh], axis=1).astype(np.float32)
    rois[-1, 3:5] = rois[-1, 1:3] - 1.0  # degenerate box: x2 < x1 -> width 1e-6
    offsets = (rng.standard_normal((R, P, 2)) * 0.3).astype(np.float32)
    return feat, rois, offsets


CASES = [
    dict(kind="roi", output_size=(1, 1), spatial_scale=1.0),
    dict(kind="roi", output_size=(1, 1), spatial_scale=0.5),
    dict(kind="roi", output_size=(2, 3), spatial_scale=1.0),   # raw bin sum (module reshape fails)
    dict(kind="ps", output_size=(1, 1), spatial_scale=1.0),
    dict(kind="ps", output_size=(2, 2), spatial_scale=0.75),
    dict(kind="ps", output_size=(2, 2), spatial_scale=1.0, part_size=(3, 3), trans_std=0.2),
    dict(kind="ps", output_size=(1, 1), spatial_scale=1.0, no_trans=True),
]


@pytest.mark.parametrize("case", CASES, ids=lambda c: "-".join(f"{k}={v}" for k, v in c.items()))
def test_roi_oracle_matches_torch_restatement(case):
    c = dict(case)
    kind = c.pop("kind")
    P = c["output_size"][0] * c["output_size"][1]
    feat, rois, offsets = roi_case(7, P=P)
    ps = kind == "ps"
    offs_t = offsets.reshape(len(rois), 2 * P) if ps else offsets
    ft = torch.tensor(feat, requires_grad=True)
    ot = torch.tensor(offs_t, requires_grad=True)
    rt_ = torch.tensor(rois)
    if ps:
        kw = dict(no_trans=c.get("no_trans", False), part_size=c.get("part_size"),
                  trans_std=c.get("trans_std", 0.1))
        out_t = torch_psroi_pool(ft, rt_, ot, c["output_size"], c["spatial_scale"], **kw)
    else:
        out_t = torch_roi_pool(ft, rt_, ot, c["output_size"], c["spatial_scale"])
    okw = dict(ps=ps, part_size=c.get("part_size"), trans_std=c.get("trans_std", 0.1),
               no_trans=c.get("no_trans", False))
    out_o = O.roi_pool_forward(feat, rois, offsets, c["output_size"], c["spatial_scale"], **okw)
    np.testing.assert_allclose(out_o, out_t.detach().numpy(), rtol=1e-5, atol=1e-5)
    g = np.random.default_rng(3).standard_normal(out_o.shape).astype(np.float32)
    out_t.backward(torch.tensor(g))
    gf, goff = O.roi_pool_backward(feat, rois, offsets, g, c["output_size"], c["spatial_scale"],
                                   **okw)
    np.testing.assert_allclose(gf, ft.grad.numpy(), rtol=1e-5, atol=1e-5)
    got = (np.zeros_like(offs_t) if ot.grad is None else ot.grad.numpy()).reshape(len(rois), P, 2)
    np.testing.assert_allclose(goff, got, rtol=1e-4, atol=1e-5)
