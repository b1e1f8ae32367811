import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "jittor-dcn_amd"), os.path.join(ROOT, "tests"), os.path.join(ROOT, "examples")]
import torch
import torch_dcn
from test_gpu_ednet import LiteralDCN, rel
dev = torch.device("cuda", 0)
B, C, O, H = 10, 16, 32, 128
torch.manual_seed(0)
a = torch_dcn.DeformConv2d(C, O, 3, 2, 1).to(dev)
with torch.no_grad():
    a.offset_conv.weight.normal_(0, 0.05); a.offset_conv.bias.uniform_(-0.5, 0.5)
sd = a.state_dict()
r64 = LiteralDCN(C, O, 3, 2, 1).double(); r64.load_state_dict({k: v.cpu().double() for k, v in sd.items()})
r32g = LiteralDCN(C, O, 3, 2, 1).to(dev); r32g.load_state_dict(sd)
x = torch.randn(B, C, H, H, device=dev)
g = None
res = {}
for name, m, xx in [("libdcn", a, x.clone()), ("lit32gpu", r32g, x.clone()), ("lit64cpu", r64, x.cpu().double())]:
    xx.requires_grad_(True)
    y = m(xx)
    if g is None:
        g = torch.randn(y.shape, device=dev)
    y.backward(g.to(y.device, y.dtype))
    res[name] = (y.detach().double().cpu(), xx.grad.double().cpu(), m.offset_conv.weight.grad.double().cpu())
for n in ("libdcn", "lit32gpu"):
    print(n, "vs f64: out", f"{rel(res[n][0], res['lit64cpu'][0]):.1e}", "gx", f"{rel(res[n][1], res['lit64cpu'][1]):.1e}", "gwo", f"{rel(res[n][2], res['lit64cpu'][2]):.1e}")
d = (res["lit32gpu"][1] - res["lit64cpu"][1]).abs()
print("max |gx| f64", float(res["lit64cpu"][1].abs().max()), "worst idx", [int(i) for i in torch.nonzero(d == d.max())[0]])
