"""Many-launch determinism and parity check of the shipped kernels, in ONE process (VERDICT r03
next item 1: the gate of DESIGN.md §4.7 — "a fused bf16 forward stays out of the product until
a build of it passes the fused_diag checks across many launches").

For each schedule it runs the full DeformConv2d step (dcn_forward + dcn_backward with
DCN_BWD_COL_IN_WS, deform_conv.py:56-81 and its autodiff) REPS times on the same resident
inputs and compares every output of every launch bit for bit with the first launch (a
transient register or LDS corruption of some lanes in some launches shows up as a
difference), and the first launch with the unfused schedule:

  config 4 (bf16, B=64, C=O=256, 28x28):
    fused   DCN_FWD_FUSED (fwd_fused_bf16<true>: the AUTO choice), columns stored: out within
            one bf16 rounding of the unfused out, every gradient bit for bit the unfused
            schedule's (its ∂W GEMM reads the stored columns, so they are K1's bits);
    nocol   DCN_FWD_FUSED_NOCOL (fwd_fused_bf16<false> + dw_fused_bf16): out bit for bit the
            fused out, every gradient but ∂W bit for bit the unfused ones, ∂W within one bf16
            rounding;
    unfused K1 + hipBLASLt (+ K5 col2im_tile, the lds_barrier users of the offset conv);
  config 3 (fp32, B=64, C=O=256, 56x56): AUTO (K1, hipBLASLt, K5, the f32 MFMA offset conv
    with its LDS-only barriers).

Device buffers are torch tensors (plumbing); every kernel is libdcn's. Prints one JSON summary
and exits 1 on any mismatch. Test infrastructure, not part of the product.

    python tools/launch_diag.py [--reps 200] [--reps3 40] [--out gpurun_out/launch_diag.json]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "jittor-dcn_amd"))

import torch  # noqa: E402

import dcn_runtime as rt  # noqa: E402


def make_case(dev, B, C, O_, H, W, bf16, seed):
    g = torch.Generator(device=dev)
    g.manual_seed(seed)
    dt = torch.bfloat16 if bf16 else torch.float32
    N, J = 9, 18
    t = {
        "x": torch.randn(B, C, H, W, device=dev, generator=g),
        "w_off": torch.randn(J, C, 3, 3, device=dev, generator=g) * (1.5 / (C * N) ** 0.5),
        "b_off": torch.rand(J, device=dev, generator=g) - 0.5,
        "w": torch.randn(O_, C, 3, 3, device=dev, generator=g) * (2.0 / (C * N)) ** 0.5,
        "b": torch.randn(O_, device=dev, generator=g) * 0.1,
        "gout": torch.randn(B, O_, H, W, device=dev, generator=g),
    }
    t = {k: v.to(dt).contiguous() for k, v in t.items()}
    desc = rt.make_desc(B, C, H, W, O_, (3, 3), (1, 1), (1, 1),
                        dtype=rt.DCN_BF16 if bf16 else rt.DCN_F32)
    wsb = rt.workspace_bytes(desc, True)
    t["ws"] = torch.empty(wsb, dtype=torch.uint8, device=dev)
    for k, shape in (("out", (B, O_, H, W)), ("off", (B, J, H, W)), ("goff", (B, J, H, W))):
        t[k] = torch.empty(shape, dtype=dt, device=dev)
    for k in ("x", "w_off", "b_off", "w", "b"):
        t["g_" + k] = torch.empty_like(t[k])
    return desc, wsb, t


def step(h, desc, wsb, t):
    P = lambda v: v.data_ptr()
    L = h.lib
    rt.check(L.dcn_forward(h.h, desc, P(t["x"]), P(t["w_off"]), P(t["b_off"]), P(t["w"]),
                           P(t["b"]), P(t["out"]), P(t["off"]), P(t["ws"]), wsb), "dcn_forward")
    rt.check(L.dcn_backward(h.h, desc, P(t["x"]), P(t["off"]), P(t["w_off"]), P(t["w"]),
                            P(t["gout"]), P(t["g_x"]), P(t["g_w"]), P(t["g_b"]), P(t["g_w_off"]),
                            P(t["g_b_off"]), P(t["goff"]), P(t["ws"]), wsb,
                            rt.DCN_BWD_COL_IN_WS), "dcn_backward")


OUTS = ("out", "off", "goff", "g_x", "g_w", "g_b", "g_w_off", "g_b_off")


def bits(v):
    return v.view(torch.int16) if v.dtype == torch.bfloat16 else v.view(torch.int32)


def within_one_bf16_ulp(a, r):
    a, r = a.double(), r.double()
    rms = float(r.pow(2).mean().sqrt())
    lim = 2.0 ** -7 * r.abs() + 2.0 ** -14 * rms
    return int(((a - r).abs() > lim).sum())


def run_schedule(h, desc, wsb, t, path, reps):
    """REPS launches; per output the launches that differ from the first, and the first."""
    h.set_fwd_path(path)
    step(h, desc, wsb, t)
    torch.cuda.synchronize()
    first = {k: t[k].clone() for k in OUTS}
    bad = {k: 0 for k in OUTS}
    bad_elems = {k: 0 for k in OUTS}
    t0 = time.perf_counter()
    for _ in range(reps - 1):
        step(h, desc, wsb, t)
        for k in OUTS:
            ne = int((bits(t[k]) != bits(first[k])).sum())
            if ne:
                bad[k] += 1
                bad_elems[k] += ne
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    h.set_fwd_path(rt.DCN_FWD_AUTO)
    return first, {"launches": reps, "launches_differing_from_first": bad,
                   "elements_differing": bad_elems, "seconds": round(el, 2)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=200)
    ap.add_argument("--reps3", type=int, default=40)
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "launch_diag.json"))
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    h = rt.Handle(0)
    h.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    res, ok = {}, True

    desc, wsb, t = make_case(dev, 64, 256, 256, 28, 28, True, 44)
    ref_u, r = run_schedule(h, desc, wsb, t, rt.DCN_FWD_UNFUSED, a.reps)
    res["config4_unfused"] = r
    ref_f, r = run_schedule(h, desc, wsb, t, rt.DCN_FWD_FUSED, a.reps)
    r["out_past_one_bf16_ulp_vs_unfused"] = within_one_bf16_ulp(ref_f["out"], ref_u["out"])
    r["tensors_not_bitwise_unfused"] = [k for k in OUTS if k != "out"
                                        and not torch.equal(bits(ref_f[k]), bits(ref_u[k]))]
    res["config4_fused_columns_stored"] = r
    ref_n, r = run_schedule(h, desc, wsb, t, rt.DCN_FWD_FUSED_NOCOL, a.reps)
    r["out_not_bitwise_fused"] = int((bits(ref_n["out"]) != bits(ref_f["out"])).sum())
    r["dW_past_one_bf16_ulp_vs_unfused"] = within_one_bf16_ulp(ref_n["g_w"], ref_u["g_w"])
    r["tensors_not_bitwise_unfused"] = [k for k in OUTS if k not in ("out", "g_w")
                                        and not torch.equal(bits(ref_n[k]), bits(ref_u[k]))]
    res["config4_fused_no_columns"] = r
    del t, ref_u, ref_f, ref_n
    torch.cuda.empty_cache()

    desc, wsb, t = make_case(dev, 64, 256, 256, 56, 56, False, 33)
    _, r = run_schedule(h, desc, wsb, t, rt.DCN_FWD_AUTO, a.reps3)
    res["config3_auto"] = r
    for name, r in res.items():
        if any(r["launches_differing_from_first"].values()):
            ok = False
        for key in ("out_past_one_bf16_ulp_vs_unfused", "out_not_bitwise_fused",
                    "dW_past_one_bf16_ulp_vs_unfused"):
            if r.get(key):
                ok = False
        if r.get("tensors_not_bitwise_unfused"):
            ok = False
    res["ok"] = ok
    res["device"] = torch.cuda.get_device_name(dev)
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res))
    h.close()
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
