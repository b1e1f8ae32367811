#!/usr/bin/env python3
"""PCIe-inclusive rate of the host-pointer API at config 3 (what the NumPy / Jittor module
calls: dcn_forward_host_s + dcn_backward_host_s on a module's host state): every step
copies x and ∂out in, out, offsets, ∂x and ∂params out. Reported beside bench.py's
HBM-resident `value`, never as it.

  python tools/host_rate.py [--chunks 0,1,4,8] [--stack 4] [--steps 5]

--chunks: image chunks of the transfer pipeline to time (0 = auto). --stack L: L modules
chained on one handle (out of one is x of the next, as EDNet stacks them, train.py:304-318),
all forwards then all backwards in reverse; ms_per_step is per module. Each backward
must reuse its own forward's state (the flags are checked)."""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "jittor-dcn_amd"))

import dcn_runtime as rt  # noqa: E402
from deform_conv import dcn_backward_numpy, dcn_forward_numpy  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--chunks", default="0")
    ap.add_argument("--stack", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    a = ap.parse_args()
    B, C, O_, H, W, k = 64, 256, 256, 56, 56, 3
    rng = np.random.default_rng(0)
    x0 = rng.standard_normal((B, C, H, W), dtype=np.float32)
    layers = []
    for _ in range(a.stack):
        wo = (rng.standard_normal((18, C, k, k)) / np.sqrt(C * 9) * 0.1).astype(np.float32)
        bo = rng.uniform(-0.5, 0.5, 18).astype(np.float32)
        w = (rng.standard_normal((O_, C, k, k)) * np.sqrt(2 / (C * 9))).astype(np.float32)
        b = (rng.standard_normal(O_) * 0.1).astype(np.float32)
        layers.append((wo, bo, w, b))
    gout = rng.standard_normal((B, O_, H, W), dtype=np.float32)
    h = rt.Handle(0)
    flags = []
    real = h.lib.dcn_backward_host_s

    def spy(*args):
        flags.append(args[-1])
        return real(*args)

    h.lib.dcn_backward_host_s = spy
    for chunks in [int(c) for c in a.chunks.split(",")]:
        states = [rt.HostState(h, chunks) for _ in layers]

        def step():
            x, ctxs = x0, []
            for st, (wo, bo, w, b) in zip(states, layers):
                out, off, ctx = dcn_forward_numpy(x, wo, bo, w, b, (1, 1), (1, 1), state=st,
                                                  return_ctx=True)
                ctxs.append((x, off, ctx))
                x = out
            g = gout
            for st, (wo, bo, w, b), (xi, off, ctx) in reversed(list(zip(states, layers, ctxs))):
                g = dcn_backward_numpy(xi, off, wo, w, True, g, (1, 1), (1, 1), ctx=ctx,
                                       offset_grad=False)["x"]

        step()
        flags.clear()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            step()
        el = (time.perf_counter() - t0) / a.steps / len(layers)
        assert flags and all(f == rt.HOST_REUSE_FWD for f in flags), flags
        print(json.dumps({"what": "host-pointer API fwd+bwd incl. PCIe, per module",
                          "chunks": chunks or "auto", "stack": len(layers),
                          "all_backwards_reused": True,
                          "staging": os.environ.get("DCN_HOST_STAGING", "0"),
                          "config": "config3", "ms_per_step": round(el * 1e3, 2),
                          "Gsamples_per_s": round(B * H * W * 9 / el / 1e9, 5)}), flush=True)
        for st in states:
            st.close()
    h.lib.dcn_backward_host_s = real
    h.close()


if __name__ == "__main__":
    main()
