import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "jittor-dcn_amd"), os.path.join(ROOT, "tests"), os.path.join(ROOT, "examples")]
import numpy as np, torch
import torch_dcn, ednet_train as E
from test_gpu_ednet import LiteralDCN
dev = torch.device("cuda", 0)
imgs, boxes, labels = E.make_data(500, 1)

def zlit(*a):
    m = LiteralDCN(*a)
    torch.nn.init.zeros_(m.offset_conv.weight); torch.nn.init.zeros_(m.offset_conv.bias)
    return m

for lib_layers in [(), (2,), (3,), (4,), (5,)]:
    torch.manual_seed(0)
    m = E.EDNet(zlit).to(dev)
    sd = m.state_dict()
    for i in lib_layers:
        name = f"conv{i}"
        old = getattr(m, name)
        new = torch_dcn.DeformConv2d(old.offset_conv.in_channels, old.weight.shape[0], 3, 2, 1).to(dev)
        new.load_state_dict(old.state_dict())
        setattr(m, name, new)
    l = E.train(m, imgs, boxes, labels, 200, log=None)
    print("libdcn layers", lib_layers, [round(float(np.mean(l[i:i + 50])), 3) for i in range(0, 200, 50)], flush=True)
