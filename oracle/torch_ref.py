"""Literal torch-CPU restatement of DeformConv2d.execute — TEST INFRASTRUCTURE ONLY.

Only tests/ (golden generation) and bench.py's cpu_baseline leg use it, as the
reference-style CPU path: the same op sequence as /root/reference/deform_conv.py:56-81
(F.conv2d for nn.Conv :58, the view/permute/arange/stack grid :62-68, normalisation by the
OUTPUT size and [norm_y, norm_x] stacking :34-39, x.repeat + grid_sample bilinear / zeros /
align_corners=True :41-52, the permutes :54 / :72 and matmul against weight.reshape(O, -1).T
:74-76, bias :79-80), with torch autograd standing in for Jittor's (train.py:414). Jittor
itself cannot be installed here; its grid_sample / Conv / matmul have these
definitions. The product path never imports this module.
"""
import torch
import torch.nn.functional as F


def literal_dcn(x, w_off, b_off, w, b, stride, padding):
    """Op-for-op restatement of deform_conv.py:56-81 (+ :30-54) in torch."""
    O, C, kh, kw = w.shape
    N = kh * kw
    B, _, H, W = x.shape
    offset = F.conv2d(x, w_off, b_off, stride=stride, padding=padding)      # :58
    H_out, W_out = offset.shape[2], offset.shape[3]                           # :59-60
    offset = offset.view(B, 2, N, H_out, W_out).permute(0, 3, 4, 2, 1)        # :62
    yv = torch.arange(H_out, dtype=x.dtype).view(1, H_out, 1, 1).repeat(B, 1, W_out, N)  # :64
    xv = torch.arange(W_out, dtype=x.dtype).view(1, 1, W_out, 1).repeat(B, H_out, 1, N)  # :65
    grid = torch.stack([xv, yv], dim=-1)                                      # :66
    coords = grid + offset                                                    # :68
    # grid_sample_wrapper (:30-54); H_out/W_out recomputed from ctor params (:34-35)
    Ho2 = (H + 2 * padding[0] - kh) // stride[0] + 1
    Wo2 = (W + 2 * padding[1] - kw) // stride[1] + 1
    norm_x = coords[..., 0] / (Wo2 - 1) * 2 - 1                               # :37
    norm_y = coords[..., 1] / (Ho2 - 1) * 2 - 1                               # :38
    g = torch.stack([norm_y, norm_x], dim=-1)                                 # :39
    x_rep = x.unsqueeze(1).repeat(1, N, 1, 1, 1).reshape(B * N, C, H, W)      # :41-42
    g = g.permute(0, 3, 1, 2, 4).reshape(B * N, Ho2, Wo2, 2)                   # :44-45
    sampled = F.grid_sample(x_rep, g, mode="bilinear", padding_mode="zeros",
                            align_corners=True)                               # :47-52
    sampled = sampled.reshape(B, N, C, Ho2, Wo2).permute(0, 2, 3, 4, 1)       # :54
    sampled = sampled.permute(0, 2, 3, 4, 1)                                  # :72
    flat = sampled.reshape(B * H_out * W_out, N * C)                          # :73
    wmat = w.reshape(O, -1).transpose(1, 0)                                   # :74
    out = torch.matmul(flat, wmat)                                            # :76
    out = out.reshape(B, H_out, W_out, O).permute(0, 3, 1, 2)                 # :77
    if b is not None:
        out = out + b.view(1, -1, 1, 1)                                       # :79-80
    return out, offset
