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
torch.manual_seed(0)
lay = torch_dcn.DeformConv2d(128, 256, 3, 2, 1).to(dev)
# step 0 with zero offsets: forward + backward (as in diag_track)
x0 = torch.randn(10, 128, 16, 16, device=dev, requires_grad=True)
y0 = lay(x0); y0.backward(torch.randn_like(y0))
lay.zero_grad()
lay.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
xt = torch.from_numpy(x).to(dev).requires_grad_(True)
y = lay(xt); torch.cuda.synchronize()
print("after fwd+bwd at zero offsets, loaded:", f"{rel(y.detach().cpu(), torch.from_numpy(ro)):.1e}")
fresh = torch_dcn.DeformConv2d(128, 256, 3, 2, 1).to(dev)
fresh.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
y2 = fresh(torch.from_numpy(x).to(dev)); torch.cuda.synchronize()
print("fresh module:", f"{rel(y2.detach().cpu(), torch.from_numpy(ro)):.1e}")
y3 = lay(torch.from_numpy(x).to(dev)); torch.cuda.synchronize()
print("lay again:", f"{rel(y3.detach().cpu(), torch.from_numpy(ro)):.1e}")
print("offset param equal:", bool(torch.equal(lay.offset_conv.weight.cpu(), fresh.offset_conv.weight.cpu())), bool(torch.equal(lay.weight.cpu(), fresh.weight.cpu())))
print("lay offset_conv.weight is contiguous:", lay.offset_conv.weight.is_contiguous(), lay.offset_conv.weight.stride(), lay.weight.stride())
