import sys, os
sys.path[:0] = ["tests", "jittor-dcn_amd", "oracle"]
import numpy as np, dcn_runtime as rt, dcn_oracle as O
import test_gpu_bf16 as T
h = rt.Handle(0)
for case in [dict(seed=1, B=2, C=64, O_=32, H=20, W=20), dict(seed=3, B=1, C=256, O_=64, H=14, W=14, off_scale=2.0)]:
    bits, v, s = T._case(**case)
    out, off, g = T._device(h, bits, s)
    _, roff, _ = O.forward(v["x"], v["w_off"], v["b_off"], v["w"], v["b"], s, (1, 1))
    ro, _, cache = O.forward(v["x"], v["w_off"], v["b_off"], v["w"], v["b"], s, (1, 1), offsets=off)
    rg = O.backward(cache, v["grad_out"])
    errs = {"off": T.rel_err(off, roff), "out": T.rel_err(out, ro)}
    for k in ("x", "weight", "bias", "offset_conv.weight", "offset_conv.bias", "offset"):
        errs[k] = T.rel_err(g[k], rg[k])
    print(case["C"], {k: f"{e:.1e}" for k, e in errs.items()})
