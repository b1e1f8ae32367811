"""Run-to-run determinism of the bf16 path at config 4 (B=64, 256->256, 28x28): fwd+bwd
three times on one handle, every tensor compared bitwise with the first run."""
import os
import sys
here = os.path.dirname(__file__)
sys.path[:0] = [os.path.join(here, "..", d) for d in ("tests", "jittor-dcn_amd", "oracle")]
import numpy as np
import dcn_runtime as rt
import test_gpu_bf16 as T

h = rt.Handle(0)
bits, v, s = T._case(75, B=64, C=256, O_=256, H=28, W=28)
ref = T._device(h, bits, s)
for run in range(2):
    got = T._device(h, bits, s)
    d = {"out": float(np.abs(got[0] - ref[0]).max()), "off": float(np.abs(got[1] - ref[1]).max())}
    d.update({k: float(np.abs(got[2][k] - ref[2][k]).max()) for k in ref[2]})
    print("run", run + 1, "vs run 0:", d, flush=True)
