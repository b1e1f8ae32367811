#!/usr/bin/env python3
"""Benchmark: DeformConv2d fwd+bwd Gsamples/s on MI355X (BASELINE.json metric).

A "step" = one DeformConv2d forward + full backward (∂x, ∂offset, ∂W, ∂b,
∂W_off, ∂b_off) over one batch of the BASELINE config-3 workload
(B=64 per GPU, C=O=256, 56×56, k=3 s=1 p=1, fp32), inputs resident in HBM, plus —
for N>1 — the RCCL all-reduce of the 631,570 parameter gradients over xGMI.
Samples per step per GPU = B·Ho·Wo·kh·kw = 1,806,336.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

One process per GPU; batch shards are independent. Default: weak scaling (B=64 images per
GPU, the driver's per-N `value`); `--global-batch G` splits a fixed batch of G images over
the N ranks instead ("scaling": "strong"; SURVEY §8(e) asks for both curves), and the
default multi-GPU run also times the fixed global batch 512 and reports it under
`strong_scaling`. value = all ranks' samples / max-over-ranks time. Rank 0 prints one JSON
line. torch is
plumbing only (HBM buffers, the stream handle, torch.distributed/RCCL); every
kernel of the step is libdcn's (hand-written gfx950 HIP + rocBLAS).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "jittor-dcn_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

METRIC = "DCN fwd+bwd Gsamples/s (N·H·W·K²/s) at N=64,C=256,56×56,k=3; 1/2/4/8 GPU"
HBM_PEAK_GBS = 8000.0  # MI355X spec (MI355X_MICROARCH.md, chip-level parameters)

CONFIGS = {
    # BASELINE.json configs[2] (config 3): the metric's own workload
    3: dict(B=64, C=256, O=256, H=56, W=56, k=3, s=1, p=1, dtype="f32"),
    # configs[3] (config 4): N=512 batch-sharded over 8 GPUs = 64 images per GPU, bf16
    4: dict(B=64, C=256, O=256, H=28, W=28, k=3, s=1, p=1, dtype="bf16"),
    # configs[0] (config 1): the reference's own CPU-runnable plumbing case, fwd+bwd
    1: dict(B=1, C=1, O=4, H=28, W=28, k=3, s=1, p=1, dtype="f32"),
    # configs[1] (config 2): forward only, vs the CPU path
    2: dict(B=8, C=64, O=128, H=56, W=56, k=3, s=1, p=1, dtype="f32", fwd_only=True),
    # configs[4] (config 5): the DCNv1 option set (extension: dilation 2, 4 deform groups;
    # parity against our own restatement only)
    5: dict(B=64, C=512, O=512, H=14, W=14, k=3, s=2, p=1, dil=2, G=4, dtype="f32"),
}


def k1_bytes(B, C, H, W, N, Ho, Wo, elem=4, J=None):
    """Algorithmic HBM bytes of one deformable-im2col launch:
    read x + read offsets (J = 2·N·deform_groups channels) + write columns."""
    J = 2 * N if J is None else J
    return elem * (B * C * H * W + B * J * Ho * Wo + B * Ho * Wo * N * C)


def shard_sizes(global_batch, world):
    """Images per rank when a fixed global batch is split over `world` ranks: as even as
    possible, the first global_batch % world ranks one image more (every rank >= 1)."""
    if global_batch < world:
        raise ValueError(f"global batch {global_batch} < {world} ranks")
    q, r = divmod(global_batch, world)
    return [q + (1 if i < r else 0) for i in range(world)]


STRONG_GLOBAL_BATCH = 512  # SURVEY §8(e) / BASELINE config 4: N=512 over 8 GPUs


def host_cpus():
    """The host cores this process may run on: the scheduler affinity mask, capped by the
    cgroup CPU quota when one is set (a GPU box shares its host; os.cpu_count() reports
    the whole machine). Returns (threads to use, description dict)."""
    ncpu = os.cpu_count() or 1
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = ncpu
    quota = None
    for path in ("/sys/fs/cgroup/cpu.max", "/sys/fs/cgroup/cpu/cpu.cfs_quota_us"):
        try:
            txt = open(path).read().split()
        except OSError:
            continue
        if path.endswith("cpu.max") and txt and txt[0] != "max":
            quota = int(txt[0]) / int(txt[1])
        elif path.endswith("cfs_quota_us") and txt and int(txt[0]) > 0:
            period = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
            quota = int(txt[0]) / period
        break
    threads = aff if quota is None else max(1, min(aff, int(quota + 0.999)))
    model = None
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return threads, {"host_threads": ncpu, "affinity_threads": aff, "cgroup_cpu_quota": quota,
                     "cpu_model": model}


def cpu_baseline(cfg, budget_s=10.0, threads=None, name="config3"):
    """Time the fp32 C restatement (oracle/dcn_ref.c, 'port') on a bounded sample:
    whole images of the configuration, fwd(+bwd), one at a time until ~budget_s, on every
    host core this process may use (host_cpus)."""
    import ref_lib as R
    R.build()
    ncpu = os.cpu_count() or 1
    auto, info = host_cpus()
    threads = threads or auto
    R.set_threads(threads)
    rng = np.random.default_rng(0)
    C, O_, H, W, k = cfg["C"], cfg["O"], cfg["H"], cfg["W"], cfg["k"]
    dil, G, fwd_only = cfg.get("dil", 1), cfg.get("G", 1), cfg.get("fwd_only", False)
    N = k * k
    x = rng.standard_normal((1, C, H, W)).astype(np.float32)
    wo = (rng.standard_normal((2 * N * G, C, k, k)) / np.sqrt(C * N)).astype(np.float32)
    bo = rng.uniform(-0.5, 0.5, 2 * N * G).astype(np.float32)
    w = (rng.standard_normal((O_, C, k, k)) * np.sqrt(2 / (C * N))).astype(np.float32)
    b = (rng.standard_normal(O_) * 0.1).astype(np.float32)
    desc = R.make_desc(x.shape, w.shape, (cfg["s"],) * 2, (cfg["p"],) * 2, (dil, dil), G)
    Ho, Wo = R.out_shape(desc)
    gout = rng.standard_normal((1, O_, Ho, Wo)).astype(np.float32)
    n_img, t0 = 0, time.perf_counter()
    while True:
        out, off = R.forward(desc, x, wo, bo, w, b)
        if not fwd_only:
            R.backward(desc, x, off, wo, w, gout)
        n_img += 1
        el = time.perf_counter() - t0
        if el >= budget_s or n_img >= 64:
            break
    samples = n_img * Ho * Wo * N
    return {"value": samples / el / 1e9, "unit": "Gsamples/s", "cores": threads, "kind": "port",
            **info,
            "sample": f"{n_img} {name} image(s) (1x{C}x{H}x{W} -> {O_}, k{k}) "
                      f"{'fwd' if fwd_only else 'fwd+bwd'}, "
                      f"oracle/dcn_ref.c fp32 OpenMP, {el:.1f} s on {threads} threads "
                      f"({info['cpu_model']}; {ncpu} host threads, "
                      f"{info['affinity_threads']} in this process's affinity mask, "
                      f"cgroup quota {info['cgroup_cpu_quota']} CPUs)"}


def cpu_baseline_framework(cfg, budget_s=10.0, threads=None, name="config3"):
    """The reference-style CPU path beside the C port: oracle/torch_ref.literal_dcn, the
    reference's own op sequence (conv, grid, x.repeat + grid_sample, permutes, matmul) on
    torch-CPU in fp32, autograd for the backward; whole images until ~budget_s. Jittor
    itself is not installable here. None where the restatement does not
    apply (dilation / deform groups)."""
    if cfg.get("dil", 1) != 1 or cfg.get("G", 1) != 1:
        return None
    import torch
    from torch_ref import literal_dcn
    ncpu = os.cpu_count() or 1
    auto, info = host_cpus()
    threads = threads or auto
    prev = torch.get_num_threads()
    torch.set_num_threads(threads)
    try:
        g = torch.Generator().manual_seed(0)
        C, O_, H, W, k = cfg["C"], cfg["O"], cfg["H"], cfg["W"], cfg["k"]
        N, st, pd = k * k, (cfg["s"],) * 2, (cfg["p"],) * 2
        fwd_only = cfg.get("fwd_only", False)
        x = torch.randn(1, C, H, W, generator=g, requires_grad=not fwd_only)
        wo = (torch.randn(2 * N, C, k, k, generator=g) / float(np.sqrt(C * N))).requires_grad_()
        bo = (torch.rand(2 * N, generator=g) - 0.5).requires_grad_()
        w = (torch.randn(O_, C, k, k, generator=g) * float(np.sqrt(2 / (C * N)))).requires_grad_()
        b = (torch.randn(O_, generator=g) * 0.1).requires_grad_()
        n_img, t0 = 0, time.perf_counter()
        while True:
            if fwd_only:
                with torch.no_grad():
                    out, _ = literal_dcn(x, wo, bo, w, b, st, pd)
            else:
                out, _ = literal_dcn(x, wo, bo, w, b, st, pd)
                out.backward(torch.ones_like(out))
            n_img += 1
            el = time.perf_counter() - t0
            if el >= budget_s or n_img >= 1024:
                break
        Ho, Wo = out.shape[2], out.shape[3]
    finally:
        torch.set_num_threads(prev)
    return {"value": n_img * Ho * Wo * N / el / 1e9, "unit": "Gsamples/s", "cores": threads,
            "kind": "port", **info,
            "sample": f"{n_img} {name} image(s) (1x{C}x{H}x{W} -> {O_}, k{k}) "
                      f"{'fwd' if fwd_only else 'fwd+bwd'}, oracle/torch_ref.py (the reference's "
                      f"op sequence, torch-CPU fp32 + autograd), {el:.1f} s on {threads} threads "
                      f"({info['cpu_model']}; {ncpu} host threads, "
                      f"{info['affinity_threads']} in this process's affinity mask, "
                      f"cgroup quota {info['cgroup_cpu_quota']} CPUs)"}


K1_KERNEL = "dcn::im2col_lds"  # K1 on the channels-last path (deform_groups 1, C % 4 == 0)


def load_traffic(path, bf16=False):
    """HBM bytes per K1 launch from the newest committed PMC summary
    (tools/pmc_pass.sh + tools/pmc_summary.py -> profiles/rNN_pmc_hbm.json); the bf16-column
    instantiation for config 4, the fp32 one otherwise."""
    import glob
    paths = [path] if path else sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_pmc_hbm.json")))
    if not paths:
        return None, None
    try:
        with open(paths[-1]) as f:
            doc = json.load(f)
    except (OSError, ValueError):
        return None, None
    for name, v in doc.get("config4" if bf16 else "kernels", {}).items():
        # bf16 K1: the 8-channel kernel (im2col_lds_b8) or the bf16 instantiation
        is_bf16 = "unsigned short" in name or name.startswith(K1_KERNEL + "_b8")
        if name.startswith(K1_KERNEL) and is_bf16 == bf16:
            return int(v["hbm_bytes"]), f"{os.path.relpath(paths[-1], ROOT)}:{name}"
    return None, None


def load_fused_traffic(bf16_cfg4_glob="r*_pmc_hbm_config4.json"):
    """HBM bytes per launch of the bf16 fused forward (columns stored) from the newest
    committed config-4 PMC summary."""
    import glob
    paths = sorted(glob.glob(os.path.join(ROOT, "profiles", bf16_cfg4_glob)))
    for path in reversed(paths):
        try:
            with open(path) as f:
                doc = json.load(f)
        except (OSError, ValueError):
            continue
        for name, v in doc.get("kernels", {}).items():
            if name.startswith("dcn::fwd_fused_bf16<true>"):
                return int(v["hbm_bytes"]), f"{os.path.relpath(path, ROOT)}:{name}"
    return None, None


def load_mfma_busy(config):
    """Counter-measured MFMA utilisation per scope (gemm_fwd, gemm_dw, gemm_dcol, offset_fwd,
    offset_bwd) from the newest committed profiles/r*_mfma_busy_config{N}.json
    (tools/pmc_mfma.sh + tools/mfma_summary.py: SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x
    GRBM_GUI_ACTIVE / 8), one rocprofv3 pass). Returns (scopes dict, relative path) or
    ({}, None)."""
    import glob
    paths = sorted(glob.glob(os.path.join(ROOT, "profiles", f"r*_mfma_busy_config{config}.json")))
    for path in reversed(paths):
        try:
            with open(path) as f:
                doc = json.load(f)
        except (OSError, ValueError):
            continue
        if doc.get("scopes"):
            return doc["scopes"], os.path.relpath(path, ROOT)
    return {}, None


def annotate_busy(entries, config):
    """Add the counter-measured MFMA utilisation beside every MFMA-bound roofline entry
    (VERDICT r05 item 3): `mfma_busy` (fraction of the matrix pipes' cycles busy while the
    kernel ran, at the clock it ran at) and `busy_source` (file:scope), in the style of
    `traffic_source`. The flop-based `frac` uses the HIP-event time and the 2.5 PF / 157.3 TF
    spec peak at its nominal clock, so the two differ by the clock the chip held (reported as
    `busy_clock_ghz`) and by MFMA work on padding."""
    scopes, src = load_mfma_busy(config)
    for e in entries or ():
        if not e or e.get("bound") != "mfma":
            continue
        sc = e.get("scope") or e["kernel"].split(" ")[0]
        v = scopes.get(sc)
        e["mfma_busy"] = v.get("mfma_busy") if v else None
        e["busy_clock_ghz"] = v.get("clock_ghz") if v else None
        e["busy_source"] = f"{src}:{sc}" if v else None
    return entries


class Workload:
    """One BASELINE configuration's replicated parameters and packed gradient buffer on
    `dev` (synthetic, SURVEY §8(d): offset conv σ = 1/sqrt(C·9) so Δ ~ N(0,1) px; the same
    seed on every rank)."""

    def __init__(self, cfg, rt, torch, dev, dcn_dp, seed=1234):
        self.cfg = cfg
        self.C, self.O, self.H, self.W = cfg["C"], cfg["O"], cfg["H"], cfg["W"]
        self.k, self.s, self.p = cfg["k"], cfg["s"], cfg["p"]
        self.dil, self.G = cfg.get("dil", 1), cfg.get("G", 1)
        self.fwd_only = cfg.get("fwd_only", False)
        self.bf16 = cfg["dtype"] == "bf16"
        self.tdt = torch.bfloat16 if self.bf16 else torch.float32
        self.N = self.k * self.k
        self.J = 2 * self.N * self.G
        self._rt = rt
        C, O_, k, N, J, tdt = self.C, self.O, self.k, self.N, self.J, self.tdt
        g = torch.Generator(device=dev)
        g.manual_seed(seed)
        self.w_off = (torch.randn(J, C, k, k, device=dev, generator=g)
                      / float(np.sqrt(C * N))).to(tdt)
        self.b_off = (torch.rand(J, device=dev, generator=g) - 0.5).to(tdt)
        self.w = (torch.randn(O_, C, k, k, device=dev, generator=g)
                  * float(np.sqrt(2.0 / (C * N)))).to(tdt)
        self.b = (torch.randn(O_, device=dev, generator=g) * 0.1).to(tdt)
        # all parameter grads packed in ONE buffer -> one all-reduce per step (dcn_dp)
        self.gbuf = dcn_dp.GradBuffer(dcn_dp.param_shapes(C, O_, k, k, deform_groups=self.G),
                                      lambda n: torch.empty(n, device=dev, dtype=tdt))
        self.gflat = self.gbuf.flat
        self.grads = tuple(self.gbuf[n] for n in dcn_dp.PARAM_ORDER)
        # ∂W and ∂b lead the packed buffer (dcn_dp.PARAM_ORDER)
        self.n_dw = self.grads[0].numel() + self.grads[1].numel()

    def desc(self, nb):
        rt = self._rt
        return rt.make_desc(nb, self.C, self.H, self.W, self.O, (self.k, self.k),
                            (self.s, self.s), (self.p, self.p), (self.dil, self.dil), self.G,
                            dtype=rt.DCN_BF16 if self.bf16 else rt.DCN_F32)


def fused_roofline(kernel_ms, B, Ho, Wo, N, C, O_):
    """The bf16 fused forward (gather + MFMA GEMM + bias, DCN_K_GEMM_FWD scope) against the
    dense bf16 MFMA peak, with its PMC traffic from the newest committed config-4 summary."""
    fl = 2.0 * B * Ho * Wo * N * C * O_
    ms = kernel_ms["gemm_fwd"]
    tr, tr_src = load_fused_traffic()
    return {
        "kernel": "dcn::fwd_fused_bf16 (f2: bilinear gather into bf16 MFMA + bias, "
                  "columns stored for the backward)",
        "bound": "mfma",
        "scope": "gemm_fwd",
        "achieved": round(fl / (ms * 1e-3) / 1e12, 1),
        "peak": 2500.0,
        "unit": "TFLOP/s",
        "frac": round(fl / (ms * 1e-3) / 1e12 / 2500.0, 4),
        "traffic": tr,
        "traffic_source": tr_src,
        "algorithmic_flop": fl,
        "avg_launch_ms": ms,
        "note": "HIP events around the launch (wf_to_frag16 swizzle included)",
    }


def config4_leg(args, world, rank, wl, rt, make_step, timed, kernel_times, fwd_path_split,
                sync):
    """BASELINE config 4 per GPU (bf16, 64 images, C=O=256, 28x28, fwd+bwd; at N > 1 with
    the gradient all-reduce) timed like `value`; returns the `config4` object of the line.
    `wl` is the config-4 Workload; `sync()` synchronises the device."""
    cfg = wl.cfg
    B = cfg["B"]
    step, bufs = make_step(wl, B, 3000 + rank)
    for _ in range(args.warmup):
        step()
    sync()
    el = timed(step, args.steps)
    km = kernel_times(step, args.steps)
    Ho, Wo = rt.out_shape(wl.desc(B))
    N, C, O_, J = wl.N, wl.C, wl.O, wl.J
    paths = (fwd_path_split(step, args.warmup, args.steps)
             if world == 1 and args.fwd_path == 0 else None)
    res = {
        "workload": f"config4: B={B}/GPU C={C}->O={O_} {cfg['H']}x{cfg['W']} k{cfg['k']} "
                    f"s{cfg['s']} p{cfg['p']} bf16 DeformConv2d fwd+bwd"
                    + (" + grad all-reduce" if world > 1 or args.exchange else ""),
        "dtype": "bf16",
        "value": round(B * world * Ho * Wo * N * args.steps / el / 1e9, 5),
        "unit": "Gsamples/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(el / args.steps * 1e3, 4),
        "scaling": "weak",
        "global_batch": B * world,
        "kernel_ms": km,
        "fwd_paths_ms_per_step": paths,
        "rooflines_other": annotate_busy(
            other_rooflines(km, B, C, O_, cfg["H"], cfg["W"], N, Ho, Wo, J, True, False)
            + [e for e in scope_rooflines(km, cfg, B, Ho, Wo)
               if e["kernel"] in ("offset_fwd", "offset_bwd")], 4),
    }
    if km.get("gemm_fwd") and not km.get("im2col"):
        res["roofline"] = annotate_busy([fused_roofline(km, B, Ho, Wo, N, C, O_)], 4)[0]
    else:  # the unfused schedule ran (K1 bf16 is the forward's HBM kernel)
        k1_ms = km.get("im2col")
        k1_b = k1_bytes(B, C, cfg["H"], cfg["W"], N, Ho, Wo, elem=2, J=J)
        ach = k1_b / (k1_ms * 1e-3) / 1e9 if k1_ms else None
        res["roofline"] = {"kernel": "dcn::im2col_lds_b8 (K1 bf16)", "bound": "hbm",
                           "achieved": round(ach, 1) if ach else None, "peak": HBM_PEAK_GBS,
                           "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4) if ach else None,
                           "algorithmic_bytes": k1_b, "avg_launch_ms": k1_ms}
    del step, bufs
    return res


def scope_rooflines(kernel_ms, cfg, B, Ho, Wo):
    """Every timed libdcn scope (DCN_K_* class, HIP-event average per call) against the
    roofline of its bound, from SURVEY §8(d)'s algorithmic work for the workload `cfg`:
    HBM bytes for the byte-moving kernels (K1, K5, transposes, bias), MFMA FLOPs for the
    contractions (the three GEMMs, the offset conv and its backward). Scope times include
    small companion launches (partial sums, swizzles), so the fractions are lower bounds.
    Returns the list, longest scope first: element 0 is the dominant kernel."""
    bf16 = cfg["dtype"] == "bf16"
    e = 2 if bf16 else 4
    C, O_, H, W, k = cfg["C"], cfg["O"], cfg["H"], cfg["W"], cfg["k"]
    N, J = k * k, 2 * k * k * cfg.get("G", 1)
    M, K = B * Ho * Wo, N * C
    peak_tf = 2500.0 if bf16 else 157.3  # dense bf16 / f32 MFMA (MI355X_MICROARCH.md)
    gemm = 2.0 * M * K * O_
    oc = 2.0 * M * K * J  # the offset conv is a k×k conv to J channels: same M, K
    work = {
        "offset_fwd": ("mfma", oc, "offset conv (K3)"),
        "im2col": ("hbm", k1_bytes(B, C, H, W, N, Ho, Wo, elem=e, J=J), "K1 deformable im2col"),
        "gemm_fwd": ("mfma", gemm, "forward GEMM (K2)"),
        "bias_fwd": ("hbm", 2 * e * B * O_ * Ho * Wo, "bias"),
        "xpose": ("hbm", 2 * e * B * C * H * W, "x -> channels-last"),
        "bwd_bias": ("hbm", 2 * e * B * O_ * Ho * Wo, "∂outT + ∂b"),
        "gemm_dw": ("mfma", gemm, "∂W GEMM (K6)"),
        "gemm_dcol": ("mfma", gemm, "∂col GEMM (K4)"),
        "col2im": ("hbm", e * (M * K + 2 * B * C * H * W + 2 * B * J * Ho * Wo),
                   "K5 col2im: ∂x and ∂offset"),
        "offset_bwd": ("mfma", 2 * oc, "offset-conv backward (K7)"),
    }
    out = []
    for name, ms in sorted(kernel_ms.items(), key=lambda kv: -kv[1]):
        if name not in work or not ms:
            continue
        bound, amount, what = work[name]
        rate = amount / (ms * 1e-3)
        if bound == "hbm":
            ach, peak, unit = rate / 1e9, HBM_PEAK_GBS, "GB/s"
        else:
            ach, peak, unit = rate / 1e12, peak_tf, "TFLOP/s"
        out.append({"kernel": name, "what": what, "bound": bound, "achieved": round(ach, 1),
                    "peak": peak, "unit": unit, "frac": round(ach / peak, 4),
                    ("algorithmic_bytes" if bound == "hbm" else "algorithmic_flop"): amount,
                    "avg_launch_ms": ms})
    return out


def extra_config_leg(num, args, wl, rt, make_step, timed, kernel_times, sync, cpu=None,
                     graph_timed=None):
    """BASELINE config 2 (fp32 forward only, B=8, 64->128, 56x56: "1xMI355X fwd only vs
    CPU") or config 5 (the DCNv1 option set, B=64, 512->512, 14x14, s2 dil2 G4, fwd+bwd) on
    one GPU, timed like `value` (warmup, barrier-free synchronize brackets: N = 1); returns
    the `config2` / `config5` object of the line: ms_per_step, value, kernel_ms, the
    dominant scope's roofline and the others, and for config 2 its own CPU baseline
    (`cpu`: the forward-only torch restatement of the reference's op sequence)."""
    cfg = wl.cfg
    B = cfg["B"]
    step, bufs = make_step(wl, B, 5000 + num)
    for _ in range(args.warmup):
        step()
    sync()
    el = timed(step, args.steps)
    km = kernel_times(step, args.steps)
    # the same step replayed from a HIP graph: these configurations are small enough that the
    # host's launch rate can set the eager step time (config 2: ≈0.09 ms of kernels), so the
    # device-side rate is reported beside it (never as this object's `value`)
    gms = graph_timed(step, args.steps) if graph_timed is not None else None
    Ho, Wo = rt.out_shape(wl.desc(B))
    N = wl.N
    roofs = scope_rooflines(km, cfg, B, Ho, Wo)
    fwd_only = cfg.get("fwd_only", False)
    value = B * Ho * Wo * N * args.steps / el / 1e9
    res = {
        "workload": f"config{num}: B={B}/GPU C={cfg['C']}->O={cfg['O']} {cfg['H']}x{cfg['W']} "
                    f"k{cfg['k']} s{cfg['s']} p{cfg['p']} dil{cfg.get('dil', 1)} "
                    f"G{cfg.get('G', 1)} {cfg['dtype']} DeformConv2d "
                    + ("fwd only" if fwd_only else "fwd+bwd"),
        "dtype": cfg["dtype"],
        "value": round(value, 5),
        "unit": "Gsamples/s",
        "n_gpus": 1,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(el / args.steps * 1e3, 4),
        "samples_per_step": B * Ho * Wo * N,
        "graph_ms_per_step": round(gms, 4) if gms else None,
        "kernel_ms": km,
        "roofline": annotate_busy(roofs[:1], num)[0] if roofs else None,
        "rooflines_other": annotate_busy(roofs[1:], num),
        "cpu_baseline": None,
    }
    if cpu is not None:
        res["cpu_baseline"] = cpu
        if cpu.get("value"):
            res["gpu_over_cpu"] = round(value / cpu["value"], 1)
    del step, bufs
    return res


MATH_NAMES = {0: "f32 MFMA (rocBLAS/hipBLASLt)", 3: "f32 via split-bf16 X3 (2 planes, opt-in)",
              6: "f32 via exact-split bf16 X6", 9: "f32 via exact-split bf16 X9"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", type=int, default=3, choices=sorted(CONFIGS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--comm", choices=("torch", "libdcn"), default="torch",
                    help="gradient all-reduce transport for N>1: torch.distributed (RCCL) or "
                         "libdcn's own RCCL communicator (dcn_allreduce_grads)")
    ap.add_argument("--math", type=int, default=0, choices=(0, 3, 6, 9),
                    help="GEMM arithmetic (include/dcn.h dcn_math): 0 native f32 MFMA, "
                         "6/9 split-bf16 fp32 (X6/X9), 3 two-plane opt-in")
    ap.add_argument("--alt-math", type=int, default=6, choices=(0, 3, 6, 9),
                    help="also time this GEMM arithmetic after the headline run (N=1, fp32 "
                         "configs; 0 = skip) and report it under 'alt'")
    ap.add_argument("--fwd-path", type=int, default=0, choices=(0, 1, 2, 3),
                    help="forward schedule (include/dcn.h dcn_fwd_path): 0 auto, 1 K1 + vendor "
                         "GEMM + bias, 2 fused im2col+GEMM where it applies")
    ap.add_argument("--graph", type=int, default=0, choices=(0, 1),
                    help="1: capture one step (libdcn launches on both of its streams, and the "
                         "all-reduce) into a HIP graph after the warmup and time its replays")
    ap.add_argument("--cpu-budget", type=float, default=10.0)
    ap.add_argument("--no-host-path", action="store_true",
                    help="skip the host-pointer API rate (PCIe-inclusive, reported beside value)")
    ap.add_argument("--traffic-json", default=None,
                    help="PMC summary (default: newest profiles/r*_pmc_hbm.json)")
    ap.add_argument("--dry", action="store_true",
                    help="launcher check without a GPU: ranks join a gloo group, sum their "
                         "rank ids and rank 0 prints the world it saw (CPU tests)")
    ap.add_argument("--global-batch", type=int, default=0,
                    help="strong scaling: split this many images over the N ranks (0: weak "
                         "scaling, the config's B per GPU)")
    ap.add_argument("--no-strong", action="store_true",
                    help="skip the secondary fixed-global-batch (512) measurement that "
                         "multi-GPU weak runs of configs 3 and 4 add under strong_scaling")
    ap.add_argument("--no-config4", action="store_true",
                    help="skip the BASELINE config-4 leg (bf16, 64 images per GPU, 28x28) that "
                         "the default config-3 run times beside the headline under `config4`")
    ap.add_argument("--no-extra-configs", action="store_true",
                    help="skip the BASELINE config-2 and config-5 legs (one GPU) that the "
                         "default config-3 run at N=1 times under `config2` / `config5`")
    ap.add_argument("--exchange", action="store_true",
                    help="run the gradient exchange even at N=1 (a 1-rank RCCL group), to "
                         "exercise the overlapped all-reduce path on one GPU")
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # `bench.py --gpus N` with no external launcher: start the N ranks here, from a
        # parent that never touches the GPU (no torch import), one process per GPU
        sys.exit(spawn_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
    if args.dry:
        return dry_run(world, rank, args.global_batch)

    # stdout carries exactly one JSON line: whatever the libraries print there (RCCL's
    # version banner at communicator init, ...) goes to stderr instead
    out_stream = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)

    import torch  # plumbing: HBM buffers, stream handle, torch.distributed (RCCL)
    import torch.distributed as dist

    import dcn_dp
    import dcn_runtime as rt

    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    exch = world > 1 or args.exchange  # gradient exchange in the step
    if exch:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29511")
        os.environ.setdefault("RANK", "0")
        os.environ.setdefault("WORLD_SIZE", "1")
        dist.init_process_group("nccl", device_id=dev)

    cfg = CONFIGS[args.config]
    B, C, O_, H, W, k, s, p = (cfg[n] for n in ("B", "C", "O", "H", "W", "k", "s", "p"))
    strong = args.global_batch > 0
    if strong:  # fixed global batch split over the ranks (SURVEY §8(e) strong scaling)
        B = shard_sizes(args.global_batch, world)[rank]
    bf16 = cfg["dtype"] == "bf16"
    N = k * k
    dil, G = cfg.get("dil", 1), cfg.get("G", 1)
    fwd_only = cfg.get("fwd_only", False)
    wl_main = Workload(cfg, rt, torch, dev, dcn_dp)
    Ho, Wo = rt.out_shape(wl_main.desc(B))
    J = 2 * N * G

    h = rt.Handle(local_rank)
    stream = torch.cuda.current_stream(dev)
    h.set_stream(stream.cuda_stream)
    h.set_math(args.math)
    h.set_fwd_path(args.fwd_path)
    L = h.lib
    P = lambda t: t.data_ptr()
    comm = None
    gs = None
    if exch and args.comm == "libdcn":
        # libdcn's own communicator attached to the handle: dcn_backward returns summed
        # gradients, the ∂W/∂b part overlapped with ∂col/col2im/offset-conv backward, the
        # sums in fp32 (bf16: over the fp32 working copies)
        uid = [dcn_dp.RcclComm.unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        comm = dcn_dp.RcclComm(h, world, rank, uid[0])
        h.set_comm(comm)
    elif exch:
        # torch.distributed (RCCL over xGMI): libdcn releases `gs` as soon as ∂W and ∂b are
        # final, so their all-reduce runs beside the rest of the backward
        gs = torch.cuda.Stream(dev)
        h.set_grad_stream(gs.cuda_stream)

    def reduce_fp32(t):
        if t.dtype == torch.float32:
            dcn_dp.allreduce_torch(t)
        else:  # bf16 gradients are summed in fp32 (one bf16 rounding of the sum)
            t32 = t.float()
            dcn_dp.allreduce_torch(t32)
            t.copy_(t32)

    def make_step(wl, nb, seed):
        """One DeformConv2d fwd + bwd (+ the gradient exchange) of workload `wl` over a
        resident shard of nb images; returns the step and the buffers it keeps alive."""
        d = wl.desc(nb)
        Ho_, Wo_ = rt.out_shape(d)
        tdt_ = wl.tdt
        gen = torch.Generator(device=dev)
        gen.manual_seed(seed)
        x = torch.randn(nb, wl.C, wl.H, wl.W, device=dev, generator=gen).to(tdt_)
        gout = torch.randn(nb, wl.O, Ho_, Wo_, device=dev, generator=gen).to(tdt_)
        out = torch.empty(nb, wl.O, Ho_, Wo_, device=dev, dtype=tdt_)
        off = torch.empty(nb, wl.J, Ho_, Wo_, device=dev, dtype=tdt_)
        gx = torch.empty_like(x)
        goff = torch.empty_like(off)
        wsb = rt.workspace_bytes(d, True)
        ws = torch.empty(wsb, dtype=torch.uint8, device=dev)
        gw, gb, gwo, gbo = wl.grads

        def step():
            rt.check(L.dcn_forward(h.h, d, P(x), P(wl.w_off), P(wl.b_off), P(wl.w), P(wl.b),
                                   P(out), P(off), P(ws), wsb), "dcn_forward")
            if wl.fwd_only:
                return
            rt.check(L.dcn_backward(h.h, d, P(x), P(off), P(wl.w_off), P(wl.w), P(gout), P(gx),
                                    P(gw), P(gb), P(gwo), P(gbo), P(goff), P(ws), wsb,
                                    rt.DCN_BWD_COL_IN_WS), "dcn_backward")
            if gs is not None:
                with torch.cuda.stream(gs):
                    # starts once ∂W/∂b are final (dcn_set_grad_stream)
                    reduce_fp32(wl.gflat[:wl.n_dw])
                reduce_fp32(wl.gflat[wl.n_dw:])  # ∂W_off/∂b_off after the whole backward
                stream.wait_stream(gs)
        return step, (x, gout, out, off, gx, goff, ws)

    def kernel_times(step, steps):
        """Average HIP-event duration per libdcn kernel class: a separate pass of `steps`
        steps with events around every launch on `stream` (outside any timed region)."""
        h.prof_enable(steps)
        for _ in range(steps):
            step()
        torch.cuda.synchronize(dev)
        km = {}
        for name in rt.KERNEL_IDS:
            tot, cnt = h.prof_read(name)
            if cnt:
                km[name] = round(tot / cnt, 4)
        h.prof_enable(0)
        return km

    def fwd_path_split(step, warmup, steps):
        """DCN_BF16: the same step under each forward schedule (include/dcn.h dcn_fwd_path),
        reported beside the headline, never as `value`."""
        res = {}
        for name, pth in (("unfused (K1 + hipBLASLt + bias)", 1),
                          ("fused, columns stored (DCN_FWD_FUSED)", 2),
                          ("fused, no column matrix (DCN_FWD_FUSED_NOCOL: recomputed dW)", 3)):
            h.set_fwd_path(pth)
            for _ in range(max(2, warmup)):
                step()
            torch.cuda.synchronize(dev)
            tp = time.perf_counter()
            for _ in range(steps):
                step()
            torch.cuda.synchronize(dev)
            res[name] = round((time.perf_counter() - tp) / steps * 1e3, 4)
        h.set_fwd_path(args.fwd_path)
        return res

    def timed(run, steps):
        """Barrier + synchronize on both sides of exactly `steps` steps; max over ranks."""
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        t0 = time.perf_counter()
        for _ in range(steps):
            run()
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        el_ = time.perf_counter() - t0
        if world > 1:
            t = torch.tensor([el_], device=dev, dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el_ = float(t.item())
        return el_

    def graph_timed(step, steps):
        """ms per replay of `step` captured into a HIP graph (libdcn bound to the capture
        stream for the capture), after two untimed replays; None if capture fails."""
        try:
            cs = torch.cuda.Stream(dev)
            cs.wait_stream(stream)
            gr = torch.cuda.CUDAGraph()
            h.set_stream(cs.cuda_stream)
            try:
                with torch.cuda.graph(gr, stream=cs):
                    step()
            finally:
                h.set_stream(stream.cuda_stream)
            for _ in range(2):
                gr.replay()
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            for _ in range(steps):
                gr.replay()
            torch.cuda.synchronize(dev)
            return (time.perf_counter() - t0) / steps * 1e3
        except Exception:  # capture unsupported here: eager only
            h.set_stream(stream.cuda_stream)
            torch.cuda.synchronize(dev)
            return None

    step, bufs = make_step(wl_main, B, 1000 + rank)
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    run = step
    graph_note = None
    if args.graph:
        # one step captured on a side stream (libdcn bound to it, its own side stream joins
        # through events); each replay is one full step of the same kernels
        try:
            # (its own name: `gs` is the gradient-exchange stream the step closes over)
            cap = torch.cuda.Stream(dev)
            cap.wait_stream(stream)
            graph = torch.cuda.CUDAGraph()
            h.set_stream(cap.cuda_stream)
            with torch.cuda.graph(graph, stream=cap):
                step()
            h.set_stream(stream.cuda_stream)
            run = graph.replay
            run()
            torch.cuda.synchronize(dev)
            graph_note = "HIP graph replay of one captured step"
        except Exception as e:  # capture unsupported: time the eager step instead
            h.set_stream(stream.cuda_stream)
            graph_note = f"graph capture failed ({type(e).__name__}: {e}); eager step timed"
            torch.cuda.synchronize(dev)
    el = timed(run, args.steps)

    # per-kernel durations: a second, separate pass of the same steps with HIP events
    # around every libdcn launch on `stream` (kept out of the timed region above)
    kernel_ms = kernel_times(step, args.steps)
    # the same step under another GEMM arithmetic (split-bf16 X6 by default), reported
    # beside the headline, never as `value`
    alt = None
    if world == 1 and not bf16 and args.alt_math and args.alt_math != args.math:
        h.prof_enable(0)  # profiling off for the timed region
        h.set_math(args.alt_math)
        for _ in range(max(2, args.warmup)):
            step()
        torch.cuda.synchronize(dev)
        ta = time.perf_counter()
        for _ in range(args.steps):
            step()
        torch.cuda.synchronize(dev)
        el_alt = time.perf_counter() - ta
        h.prof_enable(args.steps)
        for _ in range(args.steps):
            step()
        torch.cuda.synchronize(dev)
        alt_k = {}
        for name in ("gemm_fwd", "gemm_dw", "gemm_dcol"):
            tot, cnt = h.prof_read(name)
            if cnt:
                alt_k[name] = round(tot / cnt, 4)
        h.set_math(args.math)
        alt = {"gemm_math": MATH_NAMES[args.alt_math],
               "value": round(B * Ho * Wo * N * args.steps / el_alt / 1e9, 5),
               "ms_per_step": round(el_alt / args.steps * 1e3, 4), "kernel_ms": alt_k,
               "note": "same synthetic step, GEMMs in exact-split bf16 MFMA arithmetic "
                       "(DESIGN.md §4.6); reported beside the headline, not as value"}
    # DCN_BF16: the other forward schedules of the same step (include/dcn.h dcn_fwd_path),
    # timed like the alt arithmetic, reported beside the headline, never as `value`
    fwd_paths = None
    if world == 1 and bf16 and args.fwd_path == 0 and not args.graph and not fwd_only:
        fwd_paths = fwd_path_split(step, args.warmup, args.steps)
    k1_ms = kernel_ms.get("im2col")
    k1_b = k1_bytes(B, C, H, W, N, Ho, Wo, elem=2 if bf16 else 4, J=J)
    k1_name = K1_KERNEL if (G == 1 and C % 4 == 0) else "dcn::im2col_cl"

    gbatch = args.global_batch if strong else B * world
    samples = gbatch * Ho * Wo * N * args.steps
    value = samples / el / 1e9
    # the other scaling curve: a weak run of configs 3 / 4 also times the
    # fixed global batch of 512 images split over the same ranks (at N = 8 that is the weak
    # shard again); reported beside `value`, never as it
    strong_res = None
    if (not strong and not args.no_strong and args.config in (3, 4) and not fwd_only
            and not args.graph):
        h.prof_enable(0)  # no per-kernel events in this timed region
        del step, bufs, run
        torch.cuda.synchronize(dev)
        torch.cuda.empty_cache()
        shards = shard_sizes(STRONG_GLOBAL_BATCH, world)
        step2, bufs2 = make_step(wl_main, shards[rank], 2000 + rank)
        for _ in range(2):
            step2()
        st_steps = max(1, min(args.steps, 10))
        el2 = timed(step2, st_steps)
        strong_res = {
            "scaling": "strong", "global_batch": STRONG_GLOBAL_BATCH, "shards": shards,
            "steps": st_steps, "ms_per_step": round(el2 / st_steps * 1e3, 4),
            "value": round(STRONG_GLOBAL_BATCH * Ho * Wo * N * st_steps / el2 / 1e9, 5),
            "unit": "Gsamples/s",
            "note": "fixed global batch of 512 images split over the ranks, timed like value "
                    "(barrier + synchronize, max over ranks); `value` is the weak curve"}
        del step2, bufs2
        torch.cuda.empty_cache()
    # BASELINE config 4 (bf16, B = 64 per GPU, 28², the multi-GPU target's per-GPU shard)
    # beside the fp32 headline in the default run: same steps / warmup, same timed() (barrier
    # + synchronize, max over ranks; at N > 1 with the gradient all-reduce on every rank).
    # Reported under `config4`, never as `value`.
    cfg4_res = None
    if args.config == 3 and not strong and not args.no_config4 and not args.graph:
        h.prof_enable(0)
        torch.cuda.synchronize(dev)
        torch.cuda.empty_cache()
        wl4 = Workload(CONFIGS[4], rt, torch, dev, dcn_dp, seed=4321)
        cfg4_res = config4_leg(args, world, rank, wl4, rt, make_step, timed, kernel_times,
                               fwd_path_split, lambda: torch.cuda.synchronize(dev))
        del wl4
        torch.cuda.empty_cache()
    # BASELINE configs 2 and 5 (one-GPU configurations: fp32 forward only vs the CPU path, and
    # the DCNv1 option set) in the default run at N = 1, reported under `config2` /
    # `config5`, never as `value`
    extra = {}
    if (args.config == 3 and world == 1 and not strong and not args.no_extra_configs
            and not args.graph):
        for num in (2, 5):
            h.prof_enable(0)
            torch.cuda.synchronize(dev)
            torch.cuda.empty_cache()
            wlx = Workload(CONFIGS[num], rt, torch, dev, dcn_dp, seed=6000 + num)
            cpu = None
            if num == 2 and not args.no_cpu_baseline:
                cpu = cpu_baseline_framework(CONFIGS[2], min(args.cpu_budget, 8.0),
                                             name="config2")
            elif num == 5 and not args.no_cpu_baseline:
                # dilation / deform groups: the torch restatement of the reference's op
                # sequence has neither, so the C/OpenMP port (oracle/dcn_ref.c) is the baseline
                cpu = cpu_baseline(CONFIGS[5], min(args.cpu_budget, 8.0), name="config5")
            extra[num] = extra_config_leg(num, args, wlx, rt, make_step, timed, kernel_times,
                                          lambda: torch.cuda.synchronize(dev), cpu, graph_timed)
            del wlx
            torch.cuda.empty_cache()
    if rank == 0:
        achieved = k1_b / (k1_ms * 1e-3) / 1e9 if k1_ms else None
        # the committed PMC summary covers the config-3 (fp32) and config-4 (bf16) K1 only
        traffic, traffic_src = (load_traffic(args.traffic_json, bf16) if args.config in (3, 4)
                                else (None, None))
        res = {
            "metric": METRIC if args.config == 3 else
            f"DCN {'fwd' if fwd_only else 'fwd+bwd'} Gsamples/s (N·H·W·K²/s), BASELINE "
            f"config {args.config}",
            "value": round(value, 5),
            "unit": "Gsamples/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(el / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "strong" if strong else "weak",
            "vs_baseline": None,
            "dtype": cfg["dtype"],
            "gemm_math": MATH_NAMES[args.math] if not bf16 else "bf16 MFMA (fp32 accumulate)",
            "data": "synthetic",
            "config": {"workload": f"config{args.config}: B={B}/GPU C={C}->O={O_} {H}x{W} k{k} s{s} "
                                   f"p{p} dil{dil} G{G} {cfg['dtype']} DeformConv2d "
                                   + ("fwd only" if fwd_only else
                                      "fwd+bwd (+RCCL grad all-reduce if N>1)"),
                       "global_batch": gbatch,
                       "B_per_gpu": (shard_sizes(args.global_batch, world) if strong else B),
                       "C": C, "O": O_, "H": H, "W": W,
                       "kernel": k, "stride": s, "padding": p,
                       "parallelism": f"dp{world} (batch-sharded, replicated params)",
                       "grad_allreduce": (f"{args.comm} (overlapped with the backward, fp32 sums)"
                                          if exch else None)},
            "roofline": {
                "kernel": f"{k1_name} (K1, deformable bilinear im2col)",
                "bound": "hbm",
                "achieved": round(achieved, 1) if achieved else None,
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4) if achieved else None,
                "traffic": traffic,
                "traffic_source": traffic_src,
                "algorithmic_bytes": k1_b,
                "avg_launch_ms": k1_ms,
            },
            "kernel_ms": kernel_ms,
            "launch": graph_note or "eager (one launch per kernel)",
            "rooflines_other": annotate_busy(
                other_rooflines(kernel_ms, B, C, O_, H, W, N, Ho, Wo, J, bf16, fwd_only)
                + [e for e in scope_rooflines(kernel_ms, cfg, B, Ho, Wo)
                   if e["kernel"] in ("offset_fwd", "offset_bwd")], args.config),
            "alt": alt,
            "fwd_paths_ms_per_step": fwd_paths,
            "strong_scaling": strong_res,
            "config4": cfg4_res,
            "config2": extra.get(2),
            "config5": extra.get(5),
            "cpu_baseline": None,
            "cpu_baseline_other": None,
        }
        if bf16 and not k1_ms and kernel_ms.get("gemm_fwd"):
            # DCN_FWD_AUTO ran the fused forward: K1 does not exist as a
            # launch; the dominant forward kernel is the fused one (gather + GEMM + bias)
            res["roofline"] = annotate_busy([fused_roofline(kernel_ms, B, Ho, Wo, N, C, O_)],
                                            args.config)[0]
        if world == 1 and not bf16 and not args.no_host_path:
            res["host_path"] = host_path_rate(cfg, args.config)
        if world == 1 and not args.no_cpu_baseline:
            # the stronger of the two CPU restatements is the reported baseline: the
            # reference's own op sequence on torch-CPU; the C/OpenMP port rides beside it
            fw = cpu_baseline_framework(cfg, args.cpu_budget, name=f"config{args.config}")
            cport = cpu_baseline(cfg, args.cpu_budget, name=f"config{args.config}")
            res["cpu_baseline"] = fw if fw and fw["value"] >= cport["value"] else cport
            res["cpu_baseline_other"] = cport if res["cpu_baseline"] is fw else fw
        print(json.dumps(res), file=out_stream, flush=True)
    if comm is not None:
        h.set_comm(None)
        comm.close()
    h.close()
    if exch:
        dist.destroy_process_group()


def host_path_rate(cfg, config, steps=4):
    """The reference caller's path through the drop-in: DeformConv2d fwd + bwd on host (NumPy)
    arrays on a module's host state (dcn_forward_host_s + dcn_backward_host_s: persistent
    device copies, the image-chunk transfer pipeline, the backward reusing its forward's
    columns), one module and (fwd + bwd configs with C == O and stride 1) a stack of four
    (train.py:304-318: all forwards, then all backwards). PCIe-inclusive, never `value`."""
    from deform_conv import dcn_backward_numpy, dcn_forward_numpy
    import dcn_runtime as rt

    B, C, O_, H, W, k, s, p = (cfg[n] for n in ("B", "C", "O", "H", "W", "k", "s", "p"))
    if cfg.get("dil", 1) != 1 or cfg.get("G", 1) != 1:
        return None
    rng = np.random.default_rng(0)
    N = k * k
    x = rng.standard_normal((B, C, H, W), dtype=np.float32)
    wo = (rng.standard_normal((2 * N, C, k, k)) / np.sqrt(C * N)).astype(np.float32)
    bo = rng.uniform(-0.5, 0.5, 2 * N).astype(np.float32)
    w = (rng.standard_normal((O_, C, k, k)) * np.sqrt(2 / (C * N))).astype(np.float32)
    b = (rng.standard_normal(O_) * 0.1).astype(np.float32)
    h = rt.Handle(0)
    st = rt.HostState(h)  # what a DeformConv2d module holds (deform_conv.py host_state)
    Ho, Wo = rt.out_shape(rt.make_desc(B, C, H, W, O_, (k, k), (s, s), (p, p)))
    gout = rng.standard_normal((B, O_, Ho, Wo), dtype=np.float32)
    fwd_only = cfg.get("fwd_only", False)

    def step():
        out, off, ctx = dcn_forward_numpy(x, wo, bo, w, b, (s, s), (p, p), state=st,
                                          return_ctx=True)
        if not fwd_only:
            dcn_backward_numpy(x, off, wo, w, True, gout, (s, s), (p, p), ctx=ctx,
                               offset_grad=False)

    step()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    el = (time.perf_counter() - t0) / steps
    st.close()
    stack = None
    if not fwd_only and C == O_ and s == 1 and (Ho, Wo) == (H, W):
        sts = [rt.HostState(h) for _ in range(4)]

        def stack_step():
            xi, ctxs = x, []
            for sti in sts:
                o, f, c = dcn_forward_numpy(xi, wo, bo, w, b, (s, s), (p, p), state=sti,
                                            return_ctx=True)
                ctxs.append((xi, f, c))
                xi = o
            g = gout
            for xi, f, c in reversed(ctxs):
                g = dcn_backward_numpy(xi, f, wo, w, True, g, (s, s), (p, p), ctx=c,
                                       offset_grad=False)["x"]

        stack_step()
        t0 = time.perf_counter()
        for _ in range(2):
            stack_step()
        stack = round((time.perf_counter() - t0) / 2 / 4 * 1e3, 3)
        for sti in sts:
            sti.close()
    h.close()
    moved = (x.nbytes + gout.nbytes * (0 if fwd_only else 1) + B * O_ * Ho * Wo * 4
             + B * 2 * N * Ho * Wo * 4 + (0 if fwd_only else x.nbytes))
    return {"what": "host-pointer API (NumPy arrays in, NumPy arrays out) on a module's host "
                    "state: dcn_forward_host_s"
                    + ("" if fwd_only else " + dcn_backward_host_s(DCN_HOST_REUSE_FWD)")
                    + ", image-chunk transfer pipeline (auto chunks)",
            "config": f"config{config}", "steps": steps, "ms_per_step": round(el * 1e3, 3),
            "value": round(B * Ho * Wo * N / el / 1e9, 5), "unit": "Gsamples/s",
            "pcie_bytes_per_step": int(moved),
            "stack4_ms_per_module": stack,
            "transfers": "direct from / to the arrays (recycled resident outputs, hostmem.py)"
                         if os.environ.get("DCN_HOST_STAGING", "0") == "0" else
                         "pinned staging ring (DCN_HOST_STAGING=1)"}


def spawn_ranks(n):
    """Run this script once per GPU (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* in the env)
    and return the worst exit status. The parent imports nothing that touches the GPU."""
    import socket
    import subprocess
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:],
                                      env=env))
    rcs = [None] * n
    while any(rc is None for rc in rcs):
        for i, p in enumerate(procs):
            if rcs[i] is None:
                rcs[i] = p.poll()
                if rcs[i] not in (None, 0):  # one rank failed: the others would hang
                    for q in procs:
                        if q.poll() is None:
                            q.kill()
        time.sleep(0.05)
    for p in procs:
        p.wait()
    return max((abs(rc) for rc in rcs), default=0)


def dry_run(world, rank, global_batch=0):
    """--dry: the launch contract without a GPU (gloo on CPU): the ranks join one group and
    rank 0 reports the world it saw and, per rank, the images of its shard (the config's B
    per GPU, or its share of --global-batch), gathered from the ranks themselves."""
    import torch
    import torch.distributed as dist
    mine = shard_sizes(global_batch, world)[rank] if global_batch else CONFIGS[3]["B"]
    if world > 1:
        dist.init_process_group("gloo")
        t = torch.tensor([float(rank)])
        dist.all_reduce(t)
        seen = int(t.item())
        got = [torch.zeros(1) for _ in range(world)]
        dist.all_gather(got, torch.tensor([float(mine)]))
        shards = [int(v.item()) for v in got]
        dist.barrier()
        dist.destroy_process_group()
    else:
        seen, shards = 0, [mine]
    if rank == 0:
        print(json.dumps({"metric": METRIC, "value": None, "n_gpus": world, "dry": True,
                          "rank_id_sum": seen, "pid": os.getpid(),
                          "scaling": "strong" if global_batch else "weak",
                          "global_batch": sum(shards), "shards": shards}), flush=True)


def other_rooflines(kernel_ms, B, C, O_, H, W, N, Ho, Wo, J, bf16, fwd_only):
    """The other hot kernels against their bound (SURVEY §8(d) algorithmic work / the
    HIP-event scope time of the same profiled pass): the three GEMMs on the MFMA peak of
    their operand type, K5 (col2im, fp32) on HBM. Scope times include each GEMM's small
    companion launches (Σ_b partials, transposes), so these fractions are lower bounds."""
    M, K = B * Ho * Wo, N * C
    gemm_flop = 2.0 * M * K * O_
    peak_tf = 2500.0 if bf16 else 157.3  # dense bf16 / f32 MFMA (MI355X_MICROARCH.md)
    out = []
    for name in ("gemm_fwd",) + (() if fwd_only else ("gemm_dw", "gemm_dcol")):
        ms = kernel_ms.get(name)
        if ms:
            tf = gemm_flop / (ms * 1e-3) / 1e12
            out.append({"kernel": name, "bound": "mfma", "achieved": round(tf, 1),
                        "peak": peak_tf, "unit": "TFLOP/s", "frac": round(tf / peak_tf, 4),
                        "algorithmic_flop": gemm_flop, "avg_launch_ms": ms})
    ms = kernel_ms.get("gemm_dcol")
    if ms and bf16 and not fwd_only:
        # bf16 ∂columns (dcol_bf16 at config 4): a 256-deep reduction whose 231 MB of bf16
        # output outweighs its MFMA work (HBM floor 32 µs against 24 µs of MFMA at peak)
        dc_b = 2 * (M * K + M * O_ + K * O_)
        gbs = dc_b / (ms * 1e-3) / 1e9
        out.append({"kernel": "gemm_dcol (bf16 ∂columns: bytes moved)", "bound": "hbm",
                    "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": round(gbs / HBM_PEAK_GBS, 4), "algorithmic_bytes": dc_b,
                    "avg_launch_ms": ms})
    ms = kernel_ms.get("col2im")
    if ms and not bf16 and not fwd_only:
        k5_b = 4 * (M * K + 2 * B * C * H * W + 2 * B * J * Ho * Wo)
        gbs = k5_b / (ms * 1e-3) / 1e9
        out.append({"kernel": "col2im (K5: ∂x and ∂offset from ∂col)", "bound": "hbm",
                    "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": round(gbs / HBM_PEAK_GBS, 4), "algorithmic_bytes": k5_b,
                    "avg_launch_ms": ms})
    return out


if __name__ == "__main__":
    main()
