import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "jittor-dcn_amd"), os.path.join(ROOT, "tests"), os.path.join(ROOT, "examples")]
import torch, torch.nn as nn, torch.nn.functional as F
import torch_dcn
from test_gpu_ednet import LiteralDCN, rel
dev = torch.device("cuda", 0)

def run(build, inp_fn, name):
    torch.manual_seed(0)
    m1 = build(torch_dcn.DeformConv2d).to(dev)
    m64 = build(LiteralDCN).double()
    m64.load_state_dict({k: v.detach().cpu().double() for k, v in m1.state_dict().items()})
    torch.manual_seed(1)
    x = inp_fn()
    x1 = x.to(dev).requires_grad_(True); x64 = x.double().requires_grad_(True)
    y1 = m1(x1); y64 = m64(x64)
    g = torch.randn(y64.shape, dtype=torch.float64)
    y1.backward(g.to(dev, torch.float32)); y64.backward(g)
    errs = {n: f"{rel(p.grad.cpu(), dict(m64.named_parameters())[n].grad):.1e}" for n, p in m1.named_parameters()}
    print(name, "out", f"{rel(y1.cpu(), y64):.1e}", "gx", f"{rel(x1.grad.cpu(), x64.grad):.1e}", errs, flush=True)

class A(nn.Module):  # DCN only
    def __init__(s, D): super().__init__(); s.d = D(16, 32, 3, 2, 1)
    def forward(s, x): return s.d(x)
class Bm(nn.Module):  # relu -> DCN
    def __init__(s, D): super().__init__(); s.d = D(16, 32, 3, 2, 1)
    def forward(s, x): return s.d(F.relu(x))
class Cm(nn.Module):  # conv1 -> relu -> DCN
    def __init__(s, D): super().__init__(); s.c = nn.Conv2d(1, 16, 3, 1, 1); s.d = D(16, 32, 3, 2, 1)
    def forward(s, x): return s.d(F.relu(s.c(x)))
class Dm(nn.Module):  # DCN -> DCN
    def __init__(s, D): super().__init__(); s.d1 = D(16, 32, 3, 2, 1); s.d2 = D(32, 64, 3, 2, 1)
    def forward(s, x): return s.d2(F.relu(s.d1(x)))
run(A, lambda: torch.randn(10, 16, 128, 128), "dcn")
run(Bm, lambda: torch.randn(10, 16, 128, 128), "relu-dcn")
run(Cm, lambda: torch.randn(10, 1, 128, 128), "conv-relu-dcn")
run(Dm, lambda: torch.randn(10, 16, 128, 128), "dcn-dcn")
run(A, lambda: torch.randn(2, 16, 32, 32), "dcn small")
print("----")
class E1(nn.Module):  # single layer with d2's geometry
    def __init__(s, D): super().__init__(); s.d = D(32, 64, 3, 2, 1)
    def forward(s, x): return s.d(x)
run(E1, lambda: torch.randn(10, 32, 64, 64), "d2-shape alone")
run(E1, lambda: F.relu(torch.randn(10, 32, 64, 64)), "d2-shape relu input")
def mixed(first_lib):
    class M(nn.Module):
        def __init__(s, D):
            super().__init__()
            s.d1 = (D if first_lib else LiteralDCN)(16, 32, 3, 2, 1)
            s.d2 = (LiteralDCN if first_lib else D)(32, 64, 3, 2, 1)
        def forward(s, x): return s.d2(F.relu(s.d1(x)))
    return M
run(mixed(True), lambda: torch.randn(10, 16, 128, 128), "lib-then-literal")
run(mixed(False), lambda: torch.randn(10, 16, 128, 128), "literal-then-lib")
