"""SURVEY §8(f) f1 — the reference's real caller: EDNet detection training
(train.py:304-418) with libdcn DeformConv2d layers (jittor-dcn_amd/torch_dcn.py).

Parity: the same network in float64 on the CPU, with each DeformConv2d replaced by the
reference-semantics oracle (oracle/dcn_oracle.py: fp32 coordinates in the reference op
order, float64 accumulation) as a torch autograd Function. Same init, same batches:
step-0 loss and every gradient agree, and a short Adam trajectory tracks. Stride 2 at
128² -> 8², from the reference's zero offset-conv init.

Two things this test deliberately avoids, both measured in r01 (tools/diag_*.py):
  * ReLU: two correct implementations that differ by rounding take different ReLU masks
    at pre-activations within rounding of 0, and a max-norm gradient comparison through
    BatchNorm then fails on a handful of elements. The parity network uses SiLU; the
    reference ReLU network is checked by training it.
  * a float64 or fp32 *torch grid_sample* restatement as reference: their coordinate op
    order differs from the reference's fp32 one, so at floor knife edges
    their ∂offset jumps differ. The fp32 GPU one is 15 % off in ∂x on a stride-2 128²
    layer; libdcn equals the oracle to ~5e-6 there.

Tolerances: loss 1e-5 relative; every gradient max|Δ| ≤ 1e-3·max|ref|. The exception is
the conv / DeformConv2d biases that feed a train-mode BatchNorm: their exact gradient is
0, so they are checked against 1e-3 of the layer's weight-gradient scale."""
from __future__ import annotations

import os
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")
import torch.nn.functional as F  # noqa: E402

import dcn_oracle as O  # noqa: E402
import dcn_runtime as rt  # noqa: E402

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "examples"))
import ednet_train as E  # noqa: E402


class _OracleFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w_off, b_off, w, b, stride, padding):
        n = lambda t: t.detach().cpu().numpy()
        out, _, cache = O.forward(n(x), n(w_off), n(b_off), n(w), n(b), stride, padding)
        ctx.cache = cache
        return torch.from_numpy(out)

    @staticmethod
    def backward(ctx, g):
        r = O.backward(ctx.cache, g.detach().numpy())
        t = torch.from_numpy
        return (t(r["x"]), t(r["offset_conv.weight"]), t(r["offset_conv.bias"]), t(r["weight"]),
                t(r["bias"]), None, None)


class OracleDCN(torch.nn.Module):
    """DeformConv2d surface (deform_conv.py:6-28) computed by the test oracle, float64."""

    def __init__(self, cin, cout, k=3, s=1, p=1):
        super().__init__()
        self.stride, self.padding = (s, s), (p, p)
        self.offset_conv = torch.nn.Conv2d(cin, 2 * k * k, k, s, p)
        self.weight = torch.nn.Parameter(torch.zeros(cout, cin, k, k))
        self.bias = torch.nn.Parameter(torch.zeros(cout))

    def forward(self, x):
        return _OracleFn.apply(x, self.offset_conv.weight, self.offset_conv.bias, self.weight,
                               self.bias, self.stride, self.padding)


def rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))


def _nets(act):
    import torch_dcn
    torch.manual_seed(0)
    m1 = E.EDNet(torch_dcn.DeformConv2d, act=act).to("cuda")
    m64 = E.EDNet(OracleDCN, act=act).double()
    m64.load_state_dict({k: v.detach().cpu().double() for k, v in m1.state_dict().items()})
    return m1, m64


def test_ednet_step0_grads_vs_oracle():
    m1, m64 = _nets(F.silu)
    imgs, boxes, labels = E.make_data(40, seed=3)
    losses = []
    for m, dev, dt in ((m1, "cuda", torch.float32), (m64, "cpu", torch.float64)):
        xb = torch.from_numpy(imgs[:10]).to(dev, dt)
        yb = torch.from_numpy(labels[:10]).to(dev)
        bb = torch.from_numpy(boxes[:10]).to(dev, dt)
        cls, box = m(xb)
        loss = F.cross_entropy(cls, yb) + 5.0 * E.smooth_l1(box, bb)
        loss.backward()
        losses.append(loss)
    assert rel(losses[0], losses[1]) <= 1e-5
    p64 = dict(m64.named_parameters())
    for name, p in m1.named_parameters():
        ref = p64[name].grad
        if name.startswith("conv") and name.endswith(".bias") and "offset" not in name:
            scale = p64[name[:-len("bias")] + "weight"].grad.abs().max()
            err = float((p.grad.detach().cpu().double() - ref).abs().max() / scale)
        else:
            err = rel(p.grad, ref)
        assert err <= 1e-3, (name, err)


def test_ednet_adam_trajectory_vs_oracle():
    m1, m64 = _nets(F.silu)
    imgs, boxes, labels = E.make_data(40, seed=4)
    l1 = E.train(m1, imgs, boxes, labels, steps=3, seed=5, log=None)
    l64 = E.train(m64, imgs, boxes, labels, steps=3, seed=5, log=None)
    np.testing.assert_allclose(l1, l64, rtol=1e-4)


def test_ednet_relu_network_learns():
    """The reference network itself (ReLU): 300 Adam steps on the synthetic
    detection set at least halve the loss (train.py's own run: 2.42 -> 0.25 over 10
    epochs of 50 steps, README.md:824-833)."""
    import torch_dcn
    torch.manual_seed(0)
    m = E.EDNet(torch_dcn.DeformConv2d).to("cuda")
    imgs, boxes, labels = E.make_data(500, 1)
    losses = E.train(m, imgs, boxes, labels, steps=300, log=None)
    assert np.mean(losses[-50:]) < 0.5 * np.mean(losses[:20]), (losses[:5], losses[-5:])


def test_torch_stream_and_channels_last_inputs():
    """Inputs made by torch on its default stream (handle 0) right before the call, in
    channels-last memory format (what MIOpen BatchNorm hands over): libdcn must run on
    that same stream (dcn_set_stream(NULL) = the HIP null stream)."""
    import torch_dcn
    torch.manual_seed(0)
    m = torch_dcn.DeformConv2d(32, 64, 3, 2, 1).cuda()
    with torch.no_grad():
        m.offset_conv.weight.normal_(0, 0.05)
        m.offset_conv.bias.uniform_(-3, 3)
    base = torch.randn(10, 32, 40, 40, device="cuda")
    x = (base * 2.0).to(memory_format=torch.channels_last).requires_grad_(True)
    y = m(x)
    g = torch.randn_like(y)
    y.backward(g)
    sd = {k: v.detach().cpu().numpy() for k, v in m.state_dict().items()}
    xn = (base * 2.0).cpu().numpy()
    ro, _, cache = O.forward(xn, sd["offset_conv.weight"], sd["offset_conv.bias"], sd["weight"],
                             sd["bias"], (2, 2), (1, 1))
    rg = O.backward(cache, g.cpu().numpy())
    assert rel(y, torch.from_numpy(ro)) <= 1e-4
    assert rel(x.grad, torch.from_numpy(rg["x"])) <= 1e-4
    assert rel(m.offset_conv.weight.grad, torch.from_numpy(rg["offset_conv.weight"])) <= 1e-4


def test_torch_module_surface_and_bf16():
    import torch_dcn
    m = torch_dcn.DeformConv2d(16, 32, 3, 2, 1).cuda()
    assert m.kernel_size == (3, 3) and m.stride == (2, 2) and m.N == 9
    assert not m.offset_conv.weight.any() and not m.bias.any()
    x = torch.randn(2, 16, 20, 20, device="cuda")
    y = m(x)
    assert y.shape == (2, 32, 10, 10)
    mb = torch_dcn.DeformConv2d(16, 32, 3, 2, 1).cuda().to(torch.bfloat16)
    mb.load_state_dict({k: v.to(torch.bfloat16) for k, v in m.state_dict().items()})
    yb = mb(x.to(torch.bfloat16))
    assert rel(yb.float(), y) <= 1e-2
    yb.float().sum().backward()
    assert mb.weight.grad is not None and mb.weight.grad.dtype == torch.bfloat16


def test_torch_bf16_no_grad_forward_writes_no_columns():
    """A bf16 forward under torch.no_grad (the reference's jt.no_grad inference,
    train.py:430) runs dcn_forward_ex(DCN_FWD_NO_COLUMNS): same output bits as the
    grad-enabled forward (which DCN_FWD_AUTO runs fused with its columns stored when O is one
    256-channel tile and the map has at least 28 x 28 pixels), the handle's forward path is
    left as the caller set it, and the gradients of a forward followed by a no-grad forward of
    the same module stay bit for bit: the no-grad call advanced the workspace token, so the
    backward recomputes the columns."""
    import torch_dcn
    torch.manual_seed(3)
    m = torch_dcn.DeformConv2d(256, 256, 3, 1, 1).cuda().to(torch.bfloat16)
    with torch.no_grad():
        m.offset_conv.weight.normal_(0, 1.0 / 48)
        m.offset_conv.bias.uniform_(-0.5, 0.5)
    x = torch.randn(2, 256, 28, 28, device="cuda", dtype=torch.bfloat16)
    h = torch_dcn._handle(x.device)
    h.set_fwd_path(rt.DCN_FWD_FUSED)  # a path the caller chose: the no-grad call keeps it
    with torch.no_grad():
        y0 = m(x)
    assert h.get_fwd_path() == rt.DCN_FWD_FUSED
    h.set_fwd_path(rt.DCN_FWD_AUTO)
    xg = x.clone().requires_grad_(True)
    y1 = m(xg)
    assert torch.equal(y0.view(torch.int16), y1.detach().view(torch.int16))
    g = torch.randn_like(y1)
    y1.backward(g)
    gw_a = m.weight.grad.clone()
    m.weight.grad = None
    y2 = m(xg)
    with torch.no_grad():
        m(x)  # a forward-only call in between: its columns are not written
    y2.backward(g)
    assert torch.equal(gw_a.view(torch.int16), m.weight.grad.view(torch.int16))
