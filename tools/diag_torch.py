import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "jittor-dcn_amd"), os.path.join(ROOT, "tests"), os.path.join(ROOT, "examples")]
import torch
import torch_dcn
from test_gpu_ednet import LiteralDCN, rel
dev = torch.device("cuda", 0)
B, C, O, H = 10, 16, 32, 128
for mode in ["plain", "zero_ws", "sync", "no_colcache", "zero_ws+no_colcache"]:
    torch.manual_seed(0)
    a = torch_dcn.DeformConv2d(C, O, 3, 2, 1).to(dev)
    b = LiteralDCN(C, O, 3, 2, 1).to(dev)
    with torch.no_grad():
        a.offset_conv.weight.normal_(0, 0.05); a.offset_conv.bias.uniform_(-0.5, 0.5)
    b.load_state_dict(a.state_dict())
    x1 = torch.randn(B, C, H, H, device=dev, requires_grad=True)
    x2 = x1.detach().clone().requires_grad_(True)
    if "zero_ws" in mode:
        a._ws.get(1 << 30, dev).zero_()
    y1 = a(x1)
    if "no_colcache" in mode:
        a._ws.fwd_count += 1  # invalidate the cached columns -> backward recomputes
    if mode == "sync":
        torch.cuda.synchronize()
    y2 = b(x2)
    g = torch.randn_like(y1)
    y1.backward(g); y2.backward(g)
    torch.cuda.synchronize()
    print(f"{mode:20s} out {rel(y1, y2):.1e} gx {rel(x1.grad, x2.grad):.1e} gwo {rel(a.offset_conv.weight.grad, b.offset_conv.weight.grad):.1e} gw {rel(a.weight.grad, b.weight.grad):.1e}", flush=True)
# literal vs literal (torch GPU nondeterminism / sanity), and literal CPU vs literal GPU
torch.manual_seed(0)
b = LiteralDCN(C, O, 3, 2, 1).to(dev)
with torch.no_grad():
    b.offset_conv.weight.normal_(0, 0.05); b.offset_conv.bias.uniform_(-0.5, 0.5)
bc = LiteralDCN(C, O, 3, 2, 1); bc.load_state_dict({k: v.cpu() for k, v in b.state_dict().items()})
x = torch.randn(B, C, H, H, device=dev)
x2 = x.clone().requires_grad_(True); x3 = x.cpu().requires_grad_(True)
y2 = b(x2); y3 = bc(x3); g = torch.randn_like(y2)
y2.backward(g); y3.backward(g.cpu())
print("literal gpu vs cpu: out", f"{rel(y2.cpu(), y3):.1e}", "gx", f"{rel(x2.grad.cpu(), x3.grad):.1e}")
