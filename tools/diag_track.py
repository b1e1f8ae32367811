import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "jittor-dcn_amd"), os.path.join(ROOT, "tests"), os.path.join(ROOT, "examples"), os.path.join(ROOT, "oracle")]
import numpy as np, torch, torch.nn.functional as F
import torch_dcn, ednet_train as E, dcn_oracle as O
from test_gpu_ednet import LiteralDCN, rel
dev = torch.device("cuda", 0)
imgs, boxes, labels = E.make_data(500, 1)
def zlit(*a):
    m = LiteralDCN(*a); torch.nn.init.zeros_(m.offset_conv.weight); torch.nn.init.zeros_(m.offset_conv.bias); return m
torch.manual_seed(0)
m = E.EDNet(zlit).to(dev)
opt = torch.optim.Adam(m.parameters(), lr=1e-3, weight_decay=1e-4)
lay = torch_dcn.DeformConv2d(128, 256, 3, 2, 1).to(dev)
inp = {}
m.conv5.register_forward_hook(lambda mod, i, o: inp.__setitem__("x", i[0].detach()))
rng = np.random.default_rng(0)
for step in range(101):
    idx = rng.choice(500, 10, replace=False)
    xb = torch.from_numpy(imgs[idx]).to(dev); yb = torch.from_numpy(labels[idx]).to(dev); bb = torch.from_numpy(boxes[idx]).to(dev)
    opt.zero_grad()
    cls, box = m(xb)
    loss = F.cross_entropy(cls, yb) + 5 * E.smooth_l1(box, bb)
    loss.backward()
    if step % 25 == 0:
        lay.load_state_dict(m.conv5.state_dict())
        x = inp["x"]
        print("   x stride", x.stride(), "contig", x.is_contiguous(), "cl", x.is_contiguous(memory_format=torch.channels_last), x.dtype)
        with torch.no_grad():
            fr = torch_dcn.DeformConv2d(128, 256, 3, 2, 1).to(dev); fr.load_state_dict(m.conv5.state_dict())
            ya = lay(x.contiguous().clone()); yb_ = fr(x.contiguous().clone()); yc = lay(x.clone()); yd = m.conv5(x.clone())
        print("   lay(contig)", f"{rel(ya.cpu(), yd.cpu()):.1e}", "fresh(contig)", f"{rel(yb_.cpu(), yd.cpu()):.1e}", "lay(clone)", f"{rel(yc.cpu(), yd.cpu()):.1e}")
        x1 = x.clone().requires_grad_(True); x2 = x.clone().requires_grad_(True)
        y1 = lay(x1); y2 = m.conv5(x2)
        g = torch.randn_like(y1); y1.backward(g); y2.backward(g)
        sd = {k: v.detach().cpu().numpy() for k, v in m.conv5.state_dict().items()}
        ro, roff, cache = O.forward(x.cpu().numpy(), sd["offset_conv.weight"], sd["offset_conv.bias"], sd["weight"], sd["bias"], (2, 2), (1, 1))
        rg = O.backward(cache, g.cpu().numpy())
        print(step, f"loss {loss.item():.3f}", "|off|max", f"{np.abs(roff).max():.2f}",
              "lib-vs-oracle out", f"{rel(y1.detach().cpu(), torch.from_numpy(ro)):.1e}", "gx", f"{rel(x1.grad.cpu(), torch.from_numpy(rg['x'])):.1e}",
              "gw", f"{rel(lay.weight.grad.cpu(), torch.from_numpy(rg['weight'])):.1e}", "gwo", f"{rel(lay.offset_conv.weight.grad.cpu(), torch.from_numpy(rg['offset_conv.weight'])):.1e}",
              "| lit-vs-oracle out", f"{rel(y2.detach().cpu(), torch.from_numpy(ro)):.1e}", "gx", f"{rel(x2.grad.cpu(), torch.from_numpy(rg['x'])):.1e}", flush=True)
        lay.zero_grad(); m.conv5.zero_grad()
        # redo the real step's grads (they were polluted by the extra backward)
        opt.zero_grad(); cls, box = m(xb); (F.cross_entropy(cls, yb) + 5 * E.smooth_l1(box, bb)).backward()
    opt.step()
