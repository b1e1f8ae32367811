import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "jittor-dcn_amd"), os.path.join(ROOT, "tests"), os.path.join(ROOT, "examples")]
import torch, torch.nn.functional as F
import torch_dcn, ednet_train as E
from test_gpu_ednet import LiteralDCN, rel
dev = torch.device("cuda", 0)
for (B, C, O, H, zero) in [(10, 16, 32, 128, True), (10, 16, 32, 128, False), (2, 16, 32, 20, True)]:
    torch.manual_seed(0)
    a = torch_dcn.DeformConv2d(C, O, 3, 2, 1).to(dev)
    b = LiteralDCN(C, O, 3, 2, 1).to(dev)
    if not zero:
        with torch.no_grad():
            a.offset_conv.weight.normal_(0, 0.05); a.offset_conv.bias.uniform_(-0.5, 0.5)
    b.load_state_dict(a.state_dict())
    x1 = torch.randn(B, C, H, H, device=dev, requires_grad=True)
    x2 = x1.detach().clone().requires_grad_(True)
    y1, y2 = a(x1), b(x2)
    g = torch.randn_like(y1)
    y1.backward(g); y2.backward(g)
    print(B, C, O, H, "zero" if zero else "rand", "out", rel(y1, y2), "gx", rel(x1.grad, x2.grad),
          {n: round(rel(p.grad, dict(b.named_parameters())[n].grad), 6) for n, p in a.named_parameters()})
torch.manual_seed(0)
m1 = E.EDNet(torch_dcn.DeformConv2d).to(dev); m2 = E.EDNet(LiteralDCN).to(dev); m2.load_state_dict(m1.state_dict())
imgs, boxes, labels = E.make_data(40, seed=3)
xb = torch.from_numpy(imgs[:10]).to(dev); yb = torch.from_numpy(labels[:10]).to(dev); bb = torch.from_numpy(boxes[:10]).to(dev)
for m in (m1, m2):
    cls, box = m(xb); (F.cross_entropy(cls, yb) + 5.0 * E.smooth_l1(box, bb)).backward()
p2 = dict(m2.named_parameters())
for n, p in m1.named_parameters():
    print(f"{n:28s} {rel(p.grad, p2[n].grad):.2e}")
