import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "jittor-dcn_amd"), os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")]
import numpy as np, torch
import torch_dcn, dcn_oracle as O
from test_gpu_ednet import rel
dev = torch.device("cuda", 0)
z = np.load("gpurun_out/replay_conv5.npz")
sd = {"offset_conv.weight": z["offset_conv_weight"], "offset_conv.bias": z["offset_conv_bias"], "weight": z["weight"], "bias": z["bias"]}
x = z["x"]
ro, roff, _ = O.forward(x, sd["offset_conv.weight"], sd["offset_conv.bias"], sd["weight"], sd["bias"], (2, 2), (1, 1))
def check(tag, mod, xx):
    with torch.no_grad():
        y = mod(torch.from_numpy(xx).to(dev))
    torch.cuda.synchronize()
    print(tag, f"{rel(y.cpu(), torch.from_numpy(ro)):.1e}", flush=True)
a = torch_dcn.DeformConv2d(128, 256, 3, 2, 1).to(dev)
a.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
check("fresh module, 1st call", a, x)
check("same module, 2nd call", a, x)
b = torch_dcn.DeformConv2d(128, 256, 3, 2, 1).to(dev)
check("zero-offset module 1st call (ignore)", b, x)
b.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
check("after zero-offset call, loaded params", b, x)
# grad-enabled path
c = torch_dcn.DeformConv2d(128, 256, 3, 2, 1).to(dev)
c.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
xt = torch.from_numpy(x).to(dev).requires_grad_(True)
y = c(xt); torch.cuda.synchronize()
print("grad-enabled call", f"{rel(y.detach().cpu(), torch.from_numpy(ro)):.1e}")
