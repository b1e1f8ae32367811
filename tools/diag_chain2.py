import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "jittor-dcn_amd"), os.path.join(ROOT, "tests"), os.path.join(ROOT, "examples")]
import torch, torch.nn as nn, torch.nn.functional as F
import torch_dcn
from test_gpu_ednet import LiteralDCN, rel
dev = torch.device("cuda", 0)

class Dm(nn.Module):
    def __init__(s, D): super().__init__(); s.d1 = D(16, 32, 3, 2, 1); s.d2 = D(32, 64, 3, 2, 1)
    def forward(s, x):
        s.h1 = s.d1(x); s.h1.retain_grad()
        s.a1 = F.relu(s.h1); s.a1.retain_grad()
        return s.d2(s.a1)

for mode in ["default", "nocache", "sync_between"]:
    torch.manual_seed(0)
    m1 = Dm(torch_dcn.DeformConv2d).to(dev)
    m64 = Dm(LiteralDCN).double()
    m64.load_state_dict({k: v.detach().cpu().double() for k, v in m1.state_dict().items()})
    torch.manual_seed(1)
    x = torch.randn(10, 16, 128, 128)
    x1 = x.to(dev).requires_grad_(True); x64 = x.double().requires_grad_(True)
    y1 = m1(x1); y64 = m64(x64)
    if mode == "nocache":
        m1.d1._ws.fwd_count += 1; m1.d2._ws.fwd_count += 1
    g = torch.randn(y64.shape, dtype=torch.float64)
    if mode == "sync_between":
        torch.cuda.synchronize()
    y1.backward(g.to(dev, torch.float32)); y64.backward(g)
    torch.cuda.synchronize()
    print(mode, "a1 fwd", f"{rel(m1.a1.cpu(), m64.a1):.1e}", "∂a1 (d2 gx)", f"{rel(m1.a1.grad.cpu(), m64.a1.grad):.1e}",
          "∂h1", f"{rel(m1.h1.grad.cpu(), m64.h1.grad):.1e}", "gx", f"{rel(x1.grad.cpu(), x64.grad):.1e}", flush=True)
# d2 alone fed with the SAME a1 as in the chain (from f64 chain, cast)
torch.manual_seed(0)
m1 = Dm(torch_dcn.DeformConv2d).to(dev)
m64 = Dm(LiteralDCN).double(); m64.load_state_dict({k: v.detach().cpu().double() for k, v in m1.state_dict().items()})
torch.manual_seed(1)
x = torch.randn(10, 16, 128, 128)
with torch.no_grad():
    a1 = F.relu(m64.d1(x.double()))
a32 = a1.float().to(dev).requires_grad_(True); a64 = a1.clone().requires_grad_(True)
y1 = m1.d2(a32); y64 = m64.d2(a64)
g = torch.randn(y64.shape, dtype=torch.float64)
y1.backward(g.to(dev, torch.float32)); y64.backward(g)
print("d2 alone on chain a1: gx", f"{rel(a32.grad.cpu(), a64.grad):.1e}")
d = (a32.grad.cpu().double() - a64.grad).abs()
i = torch.nonzero(d == d.max())[0]
print("worst", [int(v) for v in i], float(a32.grad.cpu()[tuple(i)]), float(a64.grad[tuple(i)]), "max", float(a64.grad.abs().max()))
print("n > 1e-3 max:", int((d > 1e-3 * a64.grad.abs().max()).sum()))
