"""Config-4 determinism probe: unfused twice, fused once; max |diff| per tensor."""
import sys, os
sys.path[:0] = [os.path.join(os.path.dirname(__file__), "..", "tests"),
                os.path.join(os.path.dirname(__file__), "..", "jittor-dcn_amd"),
                os.path.join(os.path.dirname(__file__), "..", "oracle")]
import numpy as np
import dcn_runtime as rt
import test_gpu_bf16 as T

h = rt.Handle(0)
bits, v, s = T._case(75, B=64, C=256, O_=256, H=28, W=28)
runs = {}
for name, path in [("u1", rt.DCN_FWD_UNFUSED), ("u2", rt.DCN_FWD_UNFUSED), ("f", rt.DCN_FWD_FUSED),
                   ("u3", rt.DCN_FWD_UNFUSED)]:
    h.set_fwd_path(path)
    runs[name] = T._device(h, bits, s)
for a, b in [("u1", "u2"), ("u2", "u3"), ("u2", "f")]:
    oa, _, ga = runs[a]
    ob, _, gb = runs[b]
    d = {"out": float(np.abs(oa - ob).max())}
    for k in ga:
        d[k] = float(np.abs(ga[k] - gb[k]).max())
    print(a, b, d, flush=True)
gu, gf = runs["u2"][2]["weight"], runs["f"][2]["weight"]
O_ = gu.shape[0]
d = (gu != gf).reshape(O_, -1)  # flat k = n*C + c (Q5)
K = d.shape[1]
C = 256
cols = d.any(axis=0)
print("k columns differing:", int(cols.sum()), "of", K)
ks = np.nonzero(cols)[0]
print("by tap n:", np.bincount(ks // C, minlength=9).tolist())
print("by channel group of 32:", np.bincount((ks % C) // 32, minlength=8).tolist())
print("by 8-channel unit:", np.bincount((ks % 32) // 8, minlength=4).tolist())
print("rows differing:", int(d.any(axis=1).sum()))
h.set_fwd_path(rt.DCN_FWD_FUSED)
runs["f2"] = T._device(h, bits, s)
of, of2, ou = runs["f"][0], runs["f2"][0], runs["u2"][0]
print("fused out run-to-run max diff:", float(np.abs(of - of2).max()))
print("fused weight-grad run-to-run max diff:", float(np.abs(runs["f"][2]["weight"] - runs["f2"][2]["weight"]).max()))
d = np.abs(of - ou)
ulp = np.maximum(np.abs(ou), 1e-30) * 2.0 ** -7
print("out: frac differing", float((d > 0).mean()), "frac > 1 ulp", float((d > ulp).mean()), "max rel", float((d / np.maximum(np.abs(ou), 1e-3)).max()))
