"""CPU oracle for the DeformConv2d hot path — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this module, and only as the checker. The product path (jittor-dcn_amd/) never
calls it and fails loudly when the HIP library is missing.

What it restates: /root/reference/deform_conv.py:56-81 (DeformConv2d.execute)
and its Jittor autodiff, in NumPy:
  * offset conv (deform_conv.py:16-21, :58): dense conv2d, stride/padding, bias;
  * offsets viewed as [B, 2, N, Ho, Wo] (deform_conv.py:62): channel n = Δx
    (added to the column index w), channel N+n = Δy (added to the row index h);
  * base grid (w, h) with NO per-tap base offsets and NO stride (deform_conv.py:64-68);
  * normalisation by the OUTPUT size (deform_conv.py:34-38) and grid = [norm_y,
    norm_x] (deform_conv.py:39), so grid_sample(bilinear, zeros,
    align_corners=True) (deform_conv.py:47-52) reads input ROW from norm_x and
    input COLUMN from norm_y (the transposed sampling);
  * columns ordered k = n*C + c (deform_conv.py:54, :72-73) against the weight
    buffer flattened as [O][C*kh*kw] (deform_conv.py:74), i.e. W read as
    W[o][n][c] (flat index o*N*C + n*C + c);
  * bias (deform_conv.py:79-80).

Numerics: the sampling-coordinate chain is evaluated in float32 with the
reference's op order (w + Δ -> / (Wo-1) -> * 2 -> - 1 -> + 1 -> / 2 -> * (H-1)),
because which side of an integer a coordinate lands on decides the bilinear
corners and the one-sided derivative. Everything after the floor
(interpolation, GEMM, reductions, gradients) is float64.

Parity status: Jittor is not installable here, so this oracle is pinned against
a literal op-for-op torch restatement of deform_conv.py (tests/golden/
make_golden.py, torch grid_sample/conv2d/matmul in fp32 — the PyTorch-compatible
definitions Jittor's ops mirror), not against Jittor itself: "parity unpinned"
with respect to the reference runtime; see DESIGN.md §4.

Extensions (no reference oracle, BASELINE config 5): offset-conv dilation
(dil) and deform_groups G with offset channel layout [G][2][N]; channel c uses
group c // (C/G). They reduce exactly to the reference at dil=1, G=1.
"""
from __future__ import annotations

import numpy as np

F32 = np.float32


def out_size(H, W, kh, kw, sh, sw, ph, pw, dh=1, dw=1):
    """deform_conv.py:34-35 (dilation-aware for the extension)."""
    Ho = (H + 2 * ph - dh * (kh - 1) - 1) // sh + 1
    Wo = (W + 2 * pw - dw * (kw - 1) - 1) // sw + 1
    return Ho, Wo


def _pad(x, ph, pw):
    return np.pad(x, ((0, 0), (0, 0), (ph, ph), (pw, pw)))


def _patches(x, kh, kw, sh, sw, ph, pw, dh, dw, Ho, Wo):
    """x[B,C,H,W] -> P[B, C, kh, kw, Ho, Wo] (zero padding)."""
    xp = _pad(x, ph, pw)
    B, C = x.shape[:2]
    P = np.empty((B, C, kh, kw, Ho, Wo), dtype=x.dtype)
    for i in range(kh):
        for k in range(kw):
            r = i * dh
            c = k * dw
            P[:, :, i, k] = xp[:, :, r:r + sh * (Ho - 1) + 1:sh, c:c + sw * (Wo - 1) + 1:sw]
    return P


def offset_conv(x, w_off, b_off, stride, padding, dilation=(1, 1)):
    """deform_conv.py:58 — dense conv2d in float64."""
    J, C, kh, kw = w_off.shape
    H, W = x.shape[2:]
    Ho, Wo = out_size(H, W, kh, kw, *stride, *padding, *dilation)
    P = _patches(np.asarray(x, np.float64), kh, kw, *stride, *padding, *dilation, Ho, Wo)
    out = np.einsum("bcikhw,jcik->bjhw", P, np.asarray(w_off, np.float64), optimize=True)
    return out + np.asarray(b_off, np.float64)[None, :, None, None]


def sample_coords(off32, H, W, Ho, Wo, N, G):
    """fp32 coordinate chain. off32: [B, G*2*N, Ho, Wo] float32.
    Returns (iy, ix) float32 arrays [B, G, N, Ho, Wo] (iy = input row, ix = input col)."""
    B = off32.shape[0]
    o = np.asarray(off32, F32).reshape(B, G, 2, N, Ho, Wo)
    dx, dy = o[:, :, 0], o[:, :, 1]
    wv = np.arange(Wo, dtype=F32)[None, None, None, None, :]
    hv = np.arange(Ho, dtype=F32)[None, None, None, :, None]
    cx = wv + dx
    nx = cx / F32(Wo - 1)
    nx = nx * F32(2)
    nx = nx - F32(1)
    iy = ((nx + F32(1)) / F32(2)) * F32(H - 1)
    cy = hv + dy
    ny = cy / F32(Ho - 1)
    ny = ny * F32(2)
    ny = ny - F32(1)
    ix = ((ny + F32(1)) / F32(2)) * F32(W - 1)
    return iy.astype(F32), ix.astype(F32)


def _corners(iy, ix, H, W):
    r0 = np.floor(iy).astype(np.int64)
    c0 = np.floor(ix).astype(np.int64)
    fr = iy.astype(np.float64) - r0
    fc = ix.astype(np.float64) - c0
    return r0, c0, fr, fc


def _gather(xg, r, c, H, W):
    """xg: [B, Cg, H, W]; r, c: [B, N, Ho, Wo] -> vals [B, Cg, N, Ho, Wo] (0 outside)."""
    B, Cg = xg.shape[:2]
    ok = (r >= 0) & (r < H) & (c >= 0) & (c < W)
    rr = np.clip(r, 0, H - 1)
    cc = np.clip(c, 0, W - 1)
    bidx = np.arange(B)[:, None, None, None]
    v = xg[bidx, :, rr, cc]          # [B, N, Ho, Wo, Cg]
    v = np.moveaxis(v, -1, 1)        # [B, Cg, N, Ho, Wo]
    return v * ok[:, None]


def deform_sample(x, off32, Ho, Wo, N, G):
    """Columns S[B, C, N, Ho, Wo] (float64) + sampling state for backward."""
    x = np.asarray(x, np.float64)
    B, C, H, W = x.shape
    Cg = C // G
    iy, ix = sample_coords(off32, H, W, Ho, Wo, N, G)
    r0, c0, fr, fc = _corners(iy, ix, H, W)
    S = np.empty((B, C, N, Ho, Wo))
    for g in range(G):
        xg = x[:, g * Cg:(g + 1) * Cg]
        a, b_, fr_, fc_ = r0[:, g], c0[:, g], fr[:, g], fc[:, g]
        x00 = _gather(xg, a, b_, H, W)
        x01 = _gather(xg, a, b_ + 1, H, W)
        x10 = _gather(xg, a + 1, b_, H, W)
        x11 = _gather(xg, a + 1, b_ + 1, H, W)
        gr, gc = 1 - fr_, 1 - fc_
        S[:, g * Cg:(g + 1) * Cg] = (x00 * (gr * gc)[:, None] + x01 * (gr * fc_)[:, None]
                                     + x10 * (fr_ * gc)[:, None] + x11 * (fr_ * fc_)[:, None])
    return S, (iy, ix)


def weight_matrix(w):
    """deform_conv.py:74 — W[O,C,kh,kw] flattened to [O, C*kh*kw] and paired with
    columns ordered n*C + c: returns Wf[O, N, C]."""
    O, C, kh, kw = w.shape
    return np.asarray(w, np.float64).reshape(O, kh * kw, C)


def forward(x, w_off, b_off, w, b, stride, padding, dilation=(1, 1), G=1, offsets=None):
    """DeformConv2d.execute (deform_conv.py:56-81). Returns (out f64, off f32, cache).

    `offsets` (optional, fp32 [B, 2NG, Ho, Wo]) conditions everything after the offset
    conv on given offsets. ∂offset and ∂x are discontinuous where a sampling coordinate
    crosses an integer (floor), so two implementations whose offset convs round
    differently by one ulp legitimately disagree at such knife edges; the kernel
    parity tests therefore feed the device's own offsets to the oracle and check the
    offsets themselves separately."""
    O, C, kh, kw = w.shape
    N = kh * kw
    if offsets is None:
        off = offset_conv(x, w_off, b_off, stride, padding, dilation)
        off32 = off.astype(F32)  # the reference's offsets are fp32 tensors
    else:
        off32 = np.ascontiguousarray(offsets, F32)
        off = off32
    B, _, Ho, Wo = off.shape
    S, coords = deform_sample(x, off32, Ho, Wo, N, G)
    Wf = weight_matrix(w)
    out = np.einsum("bcnhw,onc->bohw", S, Wf, optimize=True)
    if b is not None:
        out = out + np.asarray(b, np.float64)[None, :, None, None]
    cache = dict(x=np.asarray(x, np.float64), off32=off32, S=S, coords=coords, w=w, w_off=w_off,
                 stride=stride, padding=padding, dilation=dilation, G=G, N=N, has_bias=b is not None)
    return out, off32, cache


def _scatter(gx, r, c, val, H, W):
    """gx[B, Cg, H, W] += val[B, Cg, N, Ho, Wo] at (r, c) [B, N, Ho, Wo], skipping OOB."""
    B, Cg = gx.shape[:2]
    ok = (r >= 0) & (r < H) & (c >= 0) & (c < W)
    bidx = np.broadcast_to(np.arange(B)[:, None, None, None], r.shape)[ok]
    rr, cc = r[ok], c[ok]
    flat = (bidx * H + rr) * W + cc                                  # [nok]
    vv = np.moveaxis(val, 1, -1)[ok]                                 # [nok, Cg]
    acc = np.zeros((B * H * W, Cg))
    np.add.at(acc, flat, vv)
    gx += acc.reshape(B, H, W, Cg).transpose(0, 3, 1, 2)


def sampling_backward(cache, dS):
    """∂x (sampling route) and ∂off from ∂S[B, C, N, Ho, Wo]."""
    x, off32, G, N = cache["x"], cache["off32"], cache["G"], cache["N"]
    B, C, H, W = x.shape
    Cg = C // G
    Ho, Wo = off32.shape[2:]
    iy, ix = cache["coords"]
    r0, c0, fr, fc = _corners(iy, ix, H, W)
    gx = np.zeros_like(x)
    goff = np.zeros((B, G, 2, N, Ho, Wo))
    sy = (H - 1) / (Wo - 1)
    sx = (W - 1) / (Ho - 1)
    for g in range(G):
        xg = x[:, g * Cg:(g + 1) * Cg]
        d = dS[:, g * Cg:(g + 1) * Cg]
        a, b_, fr_, fc_ = r0[:, g], c0[:, g], fr[:, g], fc[:, g]
        x00 = _gather(xg, a, b_, H, W)
        x01 = _gather(xg, a, b_ + 1, H, W)
        x10 = _gather(xg, a + 1, b_, H, W)
        x11 = _gather(xg, a + 1, b_ + 1, H, W)
        gr, gc = 1 - fr_, 1 - fc_
        # one-sided (right) difference: floor() has zero gradient
        d_iy = (d * ((x10 - x00) * gc[:, None] + (x11 - x01) * fc_[:, None])).sum(1)
        d_ix = (d * ((x01 - x00) * gr[:, None] + (x11 - x10) * fr_[:, None])).sum(1)
        goff[:, g, 0] = d_iy * sy
        goff[:, g, 1] = d_ix * sx
        gxg = np.zeros_like(xg)
        _scatter(gxg, a, b_, d * (gr * gc)[:, None], H, W)
        _scatter(gxg, a, b_ + 1, d * (gr * fc_)[:, None], H, W)
        _scatter(gxg, a + 1, b_, d * (fr_ * gc)[:, None], H, W)
        _scatter(gxg, a + 1, b_ + 1, d * (fr_ * fc_)[:, None], H, W)
        gx[:, g * Cg:(g + 1) * Cg] += gxg
    return gx, goff.reshape(B, G * 2 * N, Ho, Wo)


def offset_conv_backward(x, w_off, goff, stride, padding, dilation=(1, 1)):
    """Grads of deform_conv.py:58: (∂w_off, ∂b_off, ∂x contribution)."""
    x = np.asarray(x, np.float64)
    J, C, kh, kw = w_off.shape
    B, _, H, W = x.shape
    (sh, sw), (ph, pw), (dh, dw) = stride, padding, dilation
    Ho, Wo = goff.shape[2:]
    P = _patches(x, kh, kw, sh, sw, ph, pw, dh, dw, Ho, Wo)
    gw = np.einsum("bcikhw,bjhw->jcik", P, goff, optimize=True)
    gb = goff.sum(axis=(0, 2, 3))
    # ∂P[b,c,i,k,h,w] = Σ_j w_off[j,c,i,k] goff[b,j,h,w]; scatter back through the patches
    dP = np.einsum("jcik,bjhw->bcikhw", np.asarray(w_off, np.float64), goff, optimize=True)
    gxp = np.zeros((B, C, H + 2 * ph, W + 2 * pw))
    for i in range(kh):
        for k in range(kw):
            r, c = i * dh, k * dw
            gxp[:, :, r:r + sh * (Ho - 1) + 1:sh, c:c + sw * (Wo - 1) + 1:sw] += dP[:, :, i, k]
    return gw, gb, gxp[:, :, ph:ph + H, pw:pw + W]


def backward(cache, grad_out):
    """Autodiff of DeformConv2d.execute (what optimizer.backward, train.py:414, runs).
    Returns dict of float64 grads: x, weight, bias, offset_conv.weight, offset_conv.bias, offset."""
    gout = np.asarray(grad_out, np.float64)
    S, w = cache["S"], cache["w"]
    O, C, kh, kw = w.shape
    N = kh * kw
    Wf = weight_matrix(w)
    gWf = np.einsum("bohw,bcnhw->onc", gout, S, optimize=True)
    dS = np.einsum("bohw,onc->bcnhw", gout, Wf, optimize=True)
    gx, goff = sampling_backward(cache, dS)
    gwo, gbo, gx2 = offset_conv_backward(cache["x"], cache["w_off"], goff, cache["stride"],
                                         cache["padding"], cache["dilation"])
    grads = {
        "x": gx + gx2,
        "weight": gWf.reshape(O, C, kh, kw),  # flat order o*N*C + n*C + c (Q5)
        "offset_conv.weight": gwo,
        "offset_conv.bias": gbo,
        "offset": goff,
    }
    if cache["has_bias"]:
        grads["bias"] = gout.sum(axis=(0, 2, 3))
    return grads


def im2col(x, off32, kh, kw, G=1):
    """The K1 column block col[B, N*C, Ho*Wo] (k = n*C + c) in float64."""
    B, C = x.shape[:2]
    Ho, Wo = off32.shape[2:]
    N = kh * kw
    S, _ = deform_sample(x, off32, Ho, Wo, N, G)
    return S.transpose(0, 2, 1, 3, 4).reshape(B, N * C, Ho * Wo)


# ---------------------------------------------------------------------------
# Deformable RoI pooling: deform_conv.py:85-159 (DeformRoIPool) and
# :162-241 (DeformPSRoIPool). Coordinates in float32 with the reference's op order (the
# floor decides the corners); feature sums and gradients in float64. Like the reference
# (`.sum(dim=2)` at :143-157 / :239, before the reshape), the returned forward is the
# weighted corner sum over ALL bins, [R, C] or [R, C // P]; the reference's module then
# reshapes it to [R, C, ph, pw], which only succeeds for ph*pw == 1.
# ---------------------------------------------------------------------------
def roi_bins(rois, offsets, H, W, output_size, spatial_scale=1.0, ps=False, part_size=None,
             trans_std=0.1, no_trans=False):
    """Per (roi, bin): batch index, clamped corners, dx/dy, weights, offset scale."""
    f = F32
    ph, pw = output_size
    P = ph * pw
    rois = np.asarray(rois, f)
    R = rois.shape[0]
    b = np.trunc(rois[:, 0]).astype(np.int64)  # rois[:, 0].long() (:94 / :179)
    rc = rois[:, 1:5] * f(spatial_scale)  # :96 / :181
    x1, y1, x2, y2 = rc[:, 0], rc[:, 1], rc[:, 2], rc[:, 3]
    rw = np.maximum(x2 - x1, f(1e-6))  # :98-99 / :183-184
    rh = np.maximum(y2 - y1, f(1e-6))
    hg, wg = np.meshgrid(np.arange(ph, dtype=f), np.arange(pw, dtype=f), indexing="ij")
    hf, wf = hg.reshape(-1), wg.reshape(-1)  # :101-105 / :186-190
    bw_div, bh_div = (part_size[1], part_size[0]) if (ps and part_size) else (pw, ph)
    bw = rw[:, None] / f(bw_div)  # :107-108 / :191-192
    bh = rh[:, None] / f(bh_div)
    bcx = x1[:, None] + (wf + f(0.5)) * bw  # :110-111 / :194-195
    bcy = y1[:, None] + (hf + f(0.5)) * bh
    sx = np.zeros((R, P), f)
    sy = np.zeros((R, P), f)
    if not ps:  # :113-117
        o = np.asarray(offsets, f).reshape(R, P, 2)
        cx = bcx + o[:, :, 0] * rw[:, None]
        cy = bcy + o[:, :, 1] * rh[:, None]
        sx[:], sy[:] = rw[:, None], rh[:, None]
    elif not no_trans:  # :197-201
        o = np.asarray(offsets, f).reshape(R, -1)[:, :2 * P].reshape(R, P, 2)
        cx = bcx + o[:, :, 0] * rw[:, None] * f(trans_std)
        cy = bcy + o[:, :, 1] * rh[:, None] * f(trans_std)
        sx[:], sy[:] = rw[:, None] * f(trans_std), rh[:, None] * f(trans_std)
    else:
        cx, cy = bcx, bcy
    fx = np.floor(cx).astype(np.int64)
    fy = np.floor(cy).astype(np.int64)
    x0, x1c = np.clip(fx, 0, W - 1), np.clip(fx + 1, 0, W - 1)  # :121-129 / :214-222
    y0, y1c = np.clip(fy, 0, H - 1), np.clip(fy + 1, 0, H - 1)
    dx = cx - x0.astype(f)  # :131-132 / :224-225
    dy = cy - y0.astype(f)
    w = ((f(1) - dx) * (f(1) - dy), (f(1) - dx) * dy, dx * (f(1) - dy), dx * dy)  # :134-137
    return dict(b=b, corners=((y0, x0), (y1c, x0), (y0, x1c), (y1c, x1c)), dx=dx, dy=dy, w=w,
                sx=sx, sy=sy, P=P)


def _roi_channels(C, P, ps):
    """Feature channel of (output channel co, bin p): co, or co*P + p (:232-233)."""
    Cout = C // P if ps else C
    co = np.arange(Cout)[:, None]
    p = np.arange(P)[None, :]
    return Cout, (co * P + p) if ps else np.broadcast_to(co, (Cout, P))


def roi_pool_forward(features, rois, offsets, output_size, spatial_scale=1.0, ps=False,
                     part_size=None, trans_std=0.1, no_trans=False):
    feat = np.asarray(features, np.float64)
    B, C, H, W = feat.shape
    bn = roi_bins(rois, offsets, H, W, output_size, spatial_scale, ps, part_size, trans_std,
                  no_trans)
    P = bn["P"]
    Cout, ch = _roi_channels(C, P, ps)
    R = bn["b"].shape[0]
    out = np.zeros((R, Cout))
    for k in range(4):
        y, x = bn["corners"][k]
        wk = bn["w"][k].astype(np.float64)
        for r in range(R):
            v = feat[bn["b"][r]][ch, y[r][None, :], x[r][None, :]]  # [Cout, P]
            out[r] += (v * wk[r][None, :]).sum(axis=1)
    return out


def roi_pool_backward(features, rois, offsets, grad_out, output_size, spatial_scale=1.0,
                      ps=False, part_size=None, trans_std=0.1, no_trans=False):
    """(∂features [B,C,H,W], ∂offsets [R,P,2]) of roi_pool_forward (float64)."""
    feat = np.asarray(features, np.float64)
    B, C, H, W = feat.shape
    bn = roi_bins(rois, offsets, H, W, output_size, spatial_scale, ps, part_size, trans_std,
                  no_trans)
    P = bn["P"]
    Cout, ch = _roi_channels(C, P, ps)
    g = np.asarray(grad_out, np.float64).reshape(-1, Cout)
    R = g.shape[0]
    gf = np.zeros_like(feat)
    goff = np.zeros((R, P, 2))
    dx, dy = bn["dx"].astype(np.float64), bn["dy"].astype(np.float64)
    for r in range(R):
        b = bn["b"][r]
        f = [feat[b][ch, bn["corners"][k][0][r][None, :], bn["corners"][k][1][r][None, :]]
             for k in range(4)]  # each [Cout, P]
        for k in range(4):
            y, x = bn["corners"][k]
            contrib = g[r][:, None] * bn["w"][k][r].astype(np.float64)[None, :]
            np.add.at(gf[b], (ch, np.broadcast_to(y[r], ch.shape), np.broadcast_to(x[r], ch.shape)),
                      contrib)
        dcx = ((1 - dy[r]) * (f[2] - f[0]) + dy[r] * (f[3] - f[1]))  # [Cout, P]
        dcy = ((1 - dx[r]) * (f[1] - f[0]) + dx[r] * (f[3] - f[2]))
        goff[r, :, 0] = (g[r][:, None] * dcx).sum(axis=0) * bn["sx"][r]
        goff[r, :, 1] = (g[r][:, None] * dcy).sum(axis=0) * bn["sy"][r]
    return gf, goff
