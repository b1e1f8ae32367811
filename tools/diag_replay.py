import os, sys, ctypes
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "jittor-dcn_amd"), os.path.join(ROOT, "tests"), os.path.join(ROOT, "examples"), os.path.join(ROOT, "oracle")]
import numpy as np, torch, torch.nn.functional as F
import ednet_train as E, dcn_oracle as O, dcn_runtime as rt
from test_gpu_ednet import LiteralDCN, rel
import test_gpu_parity as T
dev = torch.device("cuda", 0)
imgs, boxes, labels = E.make_data(500, 1)
def zlit(*a):
    m = LiteralDCN(*a); torch.nn.init.zeros_(m.offset_conv.weight); torch.nn.init.zeros_(m.offset_conv.bias); return m
torch.manual_seed(0)
m = E.EDNet(zlit).to(dev)
opt = torch.optim.Adam(m.parameters(), lr=1e-3, weight_decay=1e-4)
inp = {}
m.conv5.register_forward_hook(lambda mod, i, o: inp.__setitem__("x", i[0].detach()))
rng = np.random.default_rng(0)
for step in range(26):
    idx = rng.choice(500, 10, replace=False)
    xb = torch.from_numpy(imgs[idx]).to(dev); yb = torch.from_numpy(labels[idx]).to(dev); bb = torch.from_numpy(boxes[idx]).to(dev)
    opt.zero_grad(); cls, box = m(xb); (F.cross_entropy(cls, yb) + 5 * E.smooth_l1(box, bb)).backward(); opt.step()
sd = {k: v.detach().cpu().numpy() for k, v in m.conv5.state_dict().items()}
x = inp["x"].cpu().numpy()
np.savez("gpurun_out/replay_conv5.npz", x=x, **{k.replace(".", "_"): v for k, v in sd.items()})
c = dict(x=x, w_off=sd["offset_conv.weight"], b_off=sd["offset_conv.bias"], w=sd["weight"], b=sd["bias"],
         grad_out=np.random.default_rng(1).standard_normal((10, 256, 8, 8)).astype(np.float32), stride=(2, 2), padding=(1, 1), dil=(1, 1), G=1)
h = rt.Handle(0)
out, off, g = T._device_fwd_bwd(h, c)
ro, roff, cache = O.forward(c["x"], c["w_off"], c["b_off"], c["w"], c["b"], (2, 2), (1, 1))
print("C-ABI offsets vs oracle", f"{rel(torch.from_numpy(off), torch.from_numpy(roff)):.1e}", "|off| max", float(np.abs(roff).max()))
ro2, _, cache2 = O.forward(c["x"], c["w_off"], c["b_off"], c["w"], c["b"], (2, 2), (1, 1), offsets=off)
print("C-ABI out vs oracle(dev offsets)", f"{rel(torch.from_numpy(out), torch.from_numpy(ro2)):.1e}")
# standalone pieces
B, C, H, W = x.shape
desc = rt.make_desc(B, C, H, W, 256, (3, 3), (2, 2), (1, 1))
D = T.Dev(h); vp = ctypes.c_void_p
px, pwo, pbo = D.up(x), D.up(c["w_off"]), D.up(c["b_off"])
poff = D.zeros(B * 18 * 64 * 4)
rt.check(h.lib.dcn_offset_conv_fwd(h.h, desc, vp(px), vp(pwo), vp(pbo), vp(poff)))
off_s = D.down(poff, (B, 18, 8, 8))
print("standalone offset conv vs oracle", f"{rel(torch.from_numpy(off_s), torch.from_numpy(roff)):.1e}")
pcol = D.zeros(B * 64 * 9 * C * 4)
rt.check(h.lib.dcn_im2col_fwd(h.h, desc, vp(px), vp(poff), vp(pcol), 0, B))
col = D.down(pcol, (B, 64, 9 * C))
rcol = O.im2col(x, off_s, 3, 3).transpose(0, 2, 1)
dd = np.abs(col - rcol)
print("im2col vs oracle", f"{float(dd.max() / np.abs(rcol).max()):.1e}", "nbad", int((dd > 1e-4).sum()), "of", dd.size)
if (dd > 1e-4).sum():
    bad = np.argwhere(dd > 1e-4)
    print("  bad imgs", np.unique(bad[:, 0]), "pixels", np.unique(bad[:, 1])[:40], "k//C (taps)", np.unique(bad[:, 2] // C), "chan", np.unique(bad[:, 2] % C)[:10])
    b0, m0, k0 = bad[0]
    n0 = k0 // C
    print("  first bad: img", b0, "pixel", m0, "tap", n0, "dx", off_s[b0, n0].reshape(-1)[m0], "dy", off_s[b0, 9 + n0].reshape(-1)[m0], "dev", col[b0, m0, k0], "ref", rcol[b0, m0, k0])
D.free()
