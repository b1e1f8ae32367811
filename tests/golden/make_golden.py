"""Generate the golden fixtures in tests/golden/*.npz.

Jittor (the reference runtime, /root/reference/deform_conv.py:1) cannot be
installed in this image, so the fixtures come from an op-for-op restatement of
DeformConv2d.execute (deform_conv.py:56-81) written with the torch primitives
whose definitions Jittor's mirror: F.conv2d for nn.Conv (:58), the same
view/permute/arange/stack grid construction (:62-68), the same normalisation by
the OUTPUT size and [norm_y, norm_x] stacking (:34-39), x.repeat + grid_sample
(bilinear, zeros, align_corners=True) (:41-52), the two permutes (:54, :72) and
matmul against weight.reshape(O, -1).T (:74-76), then bias (:79-80). Gradients
come from torch autograd (the analogue of optimizer.backward, train.py:414).

Everything runs in float32 like the reference (its fp32 rounding of the
sampling coordinates decides the bilinear corners at integer knife edges,
SURVEY Q6). A float64 twin is stored for the random-offset cases so the
oracle can also be checked beyond fp32 noise.

This script imports nothing from /root/reference. Re-run with
    python tests/golden/make_golden.py
(the fixtures are deterministic: fixed numpy seeds).
"""
from __future__ import annotations

import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle"))
from torch_ref import literal_dcn  # noqa: E402  (op-for-op restatement of :56-81)


CASES = {
    # name: (B, C, O, H, W, k, s, p, bias, offset-conv weight scale, offset-conv bias scale)
    "config1_28x28": (1, 1, 4, 28, 28, (3, 3), (1, 1), (1, 1), True, 0.6, 1.0),
    "config1_init_zero_offsets": (1, 1, 4, 28, 28, (3, 3), (1, 1), (1, 1), True, 0.0, 0.0),
    "nonsquare_stride2": (2, 3, 5, 13, 10, (3, 3), (2, 2), (1, 1), True, 0.4, 1.0),
    "large_offsets_oob": (2, 4, 3, 9, 11, (3, 3), (1, 1), (1, 1), True, 1.5, 3.0),
    "init_zero_offsets_56": (1, 2, 3, 56, 56, (3, 3), (1, 1), (1, 1), True, 0.0, 0.0),
    "k1_p0": (2, 3, 4, 8, 8, (1, 1), (1, 1), (0, 0), True, 0.5, 1.0),
    "no_bias": (2, 3, 4, 10, 9, (3, 3), (1, 1), (1, 1), False, 0.4, 1.0),
    "rect_kernel_3x2": (2, 3, 4, 11, 12, (3, 2), (1, 2), (1, 0), True, 0.4, 1.0),
    "ednet_stride2_32": (2, 4, 6, 32, 32, (3, 3), (2, 2), (1, 1), True, 0.4, 1.0),
}

FLOAT64_TWINS = {"config1_28x28", "nonsquare_stride2", "large_offsets_oob", "rect_kernel_3x2"}


def make_inputs(name, spec, seed):
    B, C, O, H, W, k, s, p, bias, wsc, bsc = spec
    rng = np.random.default_rng(seed)
    N = k[0] * k[1]
    x = rng.standard_normal((B, C, H, W)).astype(np.float32)
    w_off = (rng.standard_normal((2 * N, C, k[0], k[1])) * wsc / np.sqrt(C * N)).astype(np.float32)
    b_off = (rng.uniform(-1, 1, 2 * N) * bsc).astype(np.float32)
    std = np.sqrt(2.0 / (C * N))                                              # deform_conv.py:23
    w = (rng.standard_normal((O, C, k[0], k[1])) * std).astype(np.float32)
    b = (rng.standard_normal(O) * 0.1).astype(np.float32) if bias else None
    Ho = (H + 2 * p[0] - k[0]) // s[0] + 1
    Wo = (W + 2 * p[1] - k[1]) // s[1] + 1
    gout = rng.standard_normal((B, O, Ho, Wo)).astype(np.float32)
    return x, w_off, b_off, w, b, gout


def run(x, w_off, b_off, w, b, gout, s, p, dtype):
    t = lambda a: None if a is None else torch.tensor(a, dtype=dtype, requires_grad=True)
    tx, two, tbo, tw, tb = t(x), t(w_off), t(b_off), t(w), t(b)
    out, off = literal_dcn(tx, two, tbo, tw, tb, s, p)
    off.retain_grad()
    out.backward(torch.tensor(gout, dtype=dtype))
    B, Ho, Wo = out.shape[0], out.shape[2], out.shape[3]
    N = w.shape[2] * w.shape[3]
    # offset / its grad back to the module's [B, 2N, Ho, Wo] layout
    off_nchw = off.detach().permute(0, 4, 3, 1, 2).reshape(B, 2 * N, Ho, Wo)
    goff = off.grad.permute(0, 4, 3, 1, 2).reshape(B, 2 * N, Ho, Wo)
    res = dict(out=out.detach().numpy(), off=off_nchw.numpy(), grad_x=tx.grad.numpy(),
               grad_weight=tw.grad.numpy(), grad_offset_weight=two.grad.numpy(),
               grad_offset_bias=tbo.grad.numpy(), grad_offset=goff.numpy())
    if tb is not None:
        res["grad_bias"] = tb.grad.numpy()
    return res


def main():
    torch.set_num_threads(1)
    for i, (name, spec) in enumerate(CASES.items()):
        B, C, O, H, W, k, s, p, bias, _, _ = spec
        x, w_off, b_off, w, b, gout = make_inputs(name, spec, seed=1000 + i)
        data = dict(x=x, w_off=w_off, b_off=b_off, w=w, grad_out=gout,
                    stride=np.array(s), padding=np.array(p), kernel=np.array(k))
        if b is not None:
            data["b"] = b
        for key, val in run(x, w_off, b_off, w, b, gout, s, p, torch.float32).items():
            data["f32_" + key] = val.astype(np.float32)
        if name in FLOAT64_TWINS:
            for key, val in run(x, w_off, b_off, w, b, gout, s, p, torch.float64).items():
                data["f64_" + key] = val.astype(np.float64)
        path = os.path.join(HERE, f"{name}.npz")
        np.savez_compressed(path, **data)
        print(f"{name}: {os.path.getsize(path) / 1024:.1f} KiB")


if __name__ == "__main__":
    main()
