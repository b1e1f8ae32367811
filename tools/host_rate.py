#!/usr/bin/env python3
"""PCIe-inclusive rate of the host-pointer API (dcn_forward_host + dcn_backward_host,
what the NumPy / Jittor shim calls) at config 3: every step copies x, params and ∂out in
and out, ∂x, ∂params out. Reported beside bench.py's HBM-resident `value`, never as it."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "jittor-dcn_amd"))

from deform_conv import dcn_backward_numpy, dcn_forward_numpy  # noqa: E402


def main(steps=5):
    B, C, O_, H, W, k = 64, 256, 256, 56, 56, 3
    rng = np.random.default_rng(0)
    x = rng.standard_normal((B, C, H, W), dtype=np.float32)
    wo = (rng.standard_normal((18, C, k, k)) / np.sqrt(C * 9)).astype(np.float32)
    bo = rng.uniform(-0.5, 0.5, 18).astype(np.float32)
    w = (rng.standard_normal((O_, C, k, k)) * np.sqrt(2 / (C * 9))).astype(np.float32)
    b = (rng.standard_normal(O_) * 0.1).astype(np.float32)
    gout = rng.standard_normal((B, O_, H, W), dtype=np.float32)

    reuse = os.environ.get("HOST_REUSE", "1") != "0"

    def step():
        out, off, ctx = dcn_forward_numpy(x, wo, bo, w, b, (1, 1), (1, 1), return_ctx=True)
        dcn_backward_numpy(x, off, wo, w, True, gout, (1, 1), (1, 1), ctx=ctx if reuse else None)

    step()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    el = (time.perf_counter() - t0) / steps
    print(json.dumps({"what": "host-pointer API fwd+bwd incl. PCIe", "reuse_fwd": reuse,
                      "staging": os.environ.get("DCN_HOST_STAGING", "0"),
                      "threads": os.environ.get("DCN_HOST_THREADS", "8"),
                      "config": "config3", "ms_per_step": round(el * 1e3, 2),
                      "Gsamples_per_s": round(B * H * W * 9 / el / 1e9, 5)}))


if __name__ == "__main__":
    main()
