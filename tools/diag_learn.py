import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "jittor-dcn_amd"), os.path.join(ROOT, "tests"), os.path.join(ROOT, "examples")]
import numpy as np, torch
import torch_dcn, ednet_train as E
from test_gpu_ednet import LiteralDCN
dev = torch.device("cuda", 0)
imgs, boxes, labels = E.make_data(500, 1)
for name, D in [("literal", LiteralDCN), ("libdcn", torch_dcn.DeformConv2d)]:
    torch.manual_seed(0)
    m = E.EDNet(D).to(dev)
    if name == "literal":  # same zero offset-conv init as the reference / torch_dcn
        for mod in m.modules():
            if isinstance(mod, LiteralDCN):
                torch.nn.init.zeros_(mod.offset_conv.weight); torch.nn.init.zeros_(mod.offset_conv.bias)
    l = E.train(m, imgs, boxes, labels, 300, log=None)
    print(name, [round(float(np.mean(l[i:i + 50])), 3) for i in range(0, 300, 50)], flush=True)
