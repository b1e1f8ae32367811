import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "jittor-dcn_amd"), os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")]
import numpy as np, dcn_runtime as rt
import test_gpu_parity as T
h = rt.Handle(0)
def rel(a, b):
    return float(np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-30))
for kw in [dict(B=2, C=16, O_=32, H=128, W=128, s=(2, 2)), dict(B=10, C=16, O_=32, H=128, W=128, s=(2, 2)),
           dict(B=10, C=16, O_=32, H=64, W=64, s=(2, 2)), dict(B=10, C=16, O_=32, H=32, W=32, s=(2, 2)),
           dict(B=4, C=16, O_=32, H=128, W=128, s=(2, 2)), dict(B=2, C=16, O_=32, H=128, W=128, s=(1, 1)),
           dict(B=2, C=32, O_=32, H=96, W=96, s=(2, 2))]:
    c = T._rand_case(5, off_scale=3.0, **kw)
    out, off, g = T._device_fwd_bwd(h, c)
    ro, roff, rg = T._oracle(c, off)
    print(kw, "out", f"{rel(out, ro):.1e}", "gx", f"{rel(g['x'], rg['x']):.1e}", "goff", f"{rel(g['offset'], rg['offset']):.1e}",
          "gwo", f"{rel(g['offset_conv.weight'], rg['offset_conv.weight']):.1e}", flush=True)
    if rel(g['x'], rg['x']) > 1e-3:
        d = np.abs(g['x'] - rg['x'])
        idx = np.unravel_index(np.argmax(d), d.shape)
        bad = np.argwhere(d > 1e-3 * np.abs(rg['x']).max())
        print("   worst", idx, g['x'][idx], rg['x'][idx], "nbad", len(bad), "rows", np.unique(bad[:, 2])[:20], "cols", np.unique(bad[:, 3])[:20], "imgs", np.unique(bad[:, 0]))
