"""r03: bf16 fwd+bwd step time per forward schedule (1 unfused, 2 fused) over a few geometries,
through the torch adapter (tools-only probe; decides fused_fwd_bf16_pays)."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "jittor-dcn_amd"))
import dcn_runtime as rt  # noqa: E402
import torch_dcn  # noqa: E402

GEOS = [(64, 256, 256, 28), (64, 128, 256, 28), (64, 64, 256, 28), (32, 256, 256, 56),
        (64, 192, 256, 28), (16, 256, 512, 28)]
dev = torch.device("cuda:0")
for B, C, O, H in GEOS:
    torch.manual_seed(0)
    m = torch_dcn.DeformConv2d(C, O, 3, 1, 1).to(dev).to(torch.bfloat16)
    with torch.no_grad():
        m.offset_conv.weight.normal_(0, 1.0 / (3 * C ** 0.5))
        m.offset_conv.bias.uniform_(-0.5, 0.5)
    x = torch.randn(B, C, H, H, device=dev, dtype=torch.bfloat16, requires_grad=True)
    g = torch.randn(B, O, H, H, device=dev, dtype=torch.bfloat16)
    res = {}
    for path in (1, 2, 1, 2):
        h = torch_dcn._handle(dev)
        h.set_fwd_path(path)
        for _ in range(3):
            m(x).backward(g)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            m(x).backward(g)
        e1.record()
        torch.cuda.synchronize()
        res.setdefault(path, []).append(round(e0.elapsed_time(e1) / 20, 4))
        h.set_fwd_path(rt.DCN_FWD_AUTO)
    print(f"B={B} C={C} O={O} {H}x{H}: unfused {res[1]} ms, fused {res[2]} ms", flush=True)
