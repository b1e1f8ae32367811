import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "jittor-dcn_amd"), os.path.join(ROOT, "tests"), os.path.join(ROOT, "examples"), os.path.join(ROOT, "oracle")]
import numpy as np, torch
import torch_dcn, dcn_oracle as O
from test_gpu_ednet import LiteralDCN, rel
dev = torch.device("cuda", 0)
for (C, O_, H) in [(16, 32, 128), (32, 64, 64)]:
    torch.manual_seed(0)
    a = torch_dcn.DeformConv2d(C, O_, 3, 2, 1).to(dev)
    with torch.no_grad():
        a.offset_conv.weight.normal_(0, 0.3 / (C * 9) ** 0.5); a.offset_conv.bias.uniform_(-0.5, 0.5)
    x = torch.randn(10, C, H, H)
    x1 = x.to(dev).requires_grad_(True)
    y1 = a(x1)
    g = torch.randn(y1.shape)
    y1.backward(g.to(dev))
    # the numpy oracle (fp32 coordinates, reference op order) on the device's offsets
    sd = {k: v.detach().cpu().numpy() for k, v in a.state_dict().items()}
    xo = x.numpy()
    ro, roff, cache = O.forward(xo, sd["offset_conv.weight"], sd["offset_conv.bias"], sd["weight"], sd["bias"], (2, 2), (1, 1))
    # device offsets: recompute via a forward hook isn't exposed; compare oracle's own offsets path
    rg = O.backward(cache, g.numpy())
    gx = x1.grad.cpu().numpy()
    d = np.abs(gx - rg["x"])
    print(C, O_, H, "out", f"{rel(torch.from_numpy(y1.detach().cpu().numpy()), torch.from_numpy(ro)):.1e}",
          "gx vs oracle", f"{float(d.max() / np.abs(rg['x']).max()):.1e}", "nbad", int((d > 1e-3 * np.abs(rg['x']).max()).sum()),
          "gwo", f"{float(np.abs(a.offset_conv.weight.grad.cpu().numpy() - rg['offset_conv.weight']).max() / np.abs(rg['offset_conv.weight']).max()):.1e}", flush=True)
    if (d > 1e-3 * np.abs(rg['x']).max()).sum():
        idx = np.argwhere(d > 1e-3 * np.abs(rg['x']).max())
        print("   bad rows", np.unique(idx[:, 2])[:30], "cols", np.unique(idx[:, 3])[:30], "imgs", np.unique(idx[:, 0]), "chans", np.unique(idx[:, 1])[:20])
