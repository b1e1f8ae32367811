"""Run-to-run determinism of the fp32 path at config 3 (B=64, 256->256, 56x56): fwd+bwd
twice on the same handle, every tensor compared bitwise."""
import os
import sys
here = os.path.dirname(__file__)
sys.path[:0] = [os.path.join(here, "..", d) for d in ("tests", "jittor-dcn_amd", "oracle")]
import numpy as np
import dcn_runtime as rt
import test_gpu_parity as T

h = rt.Handle(0)
B = int(os.environ.get("DET_B", "64"))
c = T._rand_case(7, B=B, C=256, O_=256, H=56, W=56)
r1 = T._device_fwd_bwd(h, c)
r2 = T._device_fwd_bwd(h, c)
print("out", float(np.abs(r1[0] - r2[0]).max()), "off", float(np.abs(r1[1] - r2[1]).max()))
for k in r1[2]:
    print(k, float(np.abs(r1[2][k] - r2[2][k]).max()), flush=True)
