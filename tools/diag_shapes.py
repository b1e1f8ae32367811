import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "jittor-dcn_amd"), os.path.join(ROOT, "tests"), os.path.join(ROOT, "examples")]
import torch, torch.nn as nn
import torch_dcn
from test_gpu_ednet import LiteralDCN, rel
dev = torch.device("cuda", 0)
for (C, O, H) in [(16, 32, 128), (32, 64, 64), (64, 128, 32), (128, 256, 16)]:
    for rnd in (False, True):
        torch.manual_seed(0)
        a = torch_dcn.DeformConv2d(C, O, 3, 2, 1).to(dev)
        if rnd:
            with torch.no_grad():
                a.offset_conv.weight.normal_(0, 0.3 / (C * 9) ** 0.5); a.offset_conv.bias.uniform_(-0.5, 0.5)
        r = LiteralDCN(C, O, 3, 2, 1).double(); r.load_state_dict({k: v.cpu().double() for k, v in a.state_dict().items()})
        x = torch.randn(10, C, H, H)
        x1 = x.to(dev).requires_grad_(True); x64 = x.double().requires_grad_(True)
        y1 = a(x1); y64 = r(x64)
        g = torch.randn(y64.shape, dtype=torch.float64)
        y1.backward(g.to(dev, torch.float32)); y64.backward(g)
        pr = dict(r.named_parameters())
        print(C, O, H, "rand" if rnd else "zero", "out", f"{rel(y1.cpu(), y64):.1e}", "gx", f"{rel(x1.grad.cpu(), x64.grad):.1e}",
              {n: f"{rel(p.grad.cpu(), pr[n].grad):.1e}" for n, p in a.named_parameters()}, flush=True)
