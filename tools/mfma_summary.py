#!/usr/bin/env python3
"""Per-kernel and per-scope MFMA utilisation from a tools/pmc_mfma.sh pass.

    mfma_summary.py DIR OUT_JSON --config N

Counters (rocprofv3 sums each over the whole device per dispatch; rocprofv3 serialises the
dispatches of a counter pass, so each row is one kernel alone on the chip):
  SQ_VALU_MFMA_BUSY_CYCLES  matrix-pipe busy cycles, summed over SIMDs (MI355X_MICROARCH.md:
                            "= 32 x N_mfma for 32x32x16 bf16", i.e. the per-SIMD issue cycles of
                            each MFMA: 16 for 16x16x32 bf16, 32 for 16x16x4 f32, 64 for 32x32x2 f32)
  GRBM_GUI_ACTIVE           GPU-active cycles summed over the 8 XCDs (guide, "DVFS give-back")
  SQ_BUSY_CYCLES, SQ_WAVE_CYCLES  kept for reference

Derived per dispatch:
  mfma_busy      = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x 2.4 GHz x duration): the fraction of
                   the chip's peak MFMA issue capacity the kernel used (duration from the kernel
                   trace of the same pass) -- comparable with bench.py's flop-based `frac`, except
                   that it counts the MFMAs actually issued (padding included)
  cycles         = GRBM_GUI_ACTIVE / 8; clock_ghz = cycles / duration; mfma_busy_gui = busy /
                   (1024 x cycles): the same at the clock the counters saw. GRBM_GUI_ACTIVE also
                   counts the dispatch's ramp, so on kernels of tens of µs clock_ghz reads above
                   the 2.4 GHz peak and mfma_busy_gui low; mfma_busy is the one reported
A scope (a bench.py kernel_ms class: gemm_fwd, gemm_dw, ...) is the busy-cycle-weighted union
of its kernels: sum(busy) / (1024 x 2.4 GHz x sum(duration)).
Calibration (config 4): fwd_fused_bf16<true> issues exactly 512 x 4 x 72 x 28 16x16x32 bf16
MFMAs; the counter reads 16 cycles per MFMA of it (ratio 1.0000 in profiles/r06a_*).

hipBLASLt / rocBLAS GEMM kernels (Cijk_*) are attributed to scopes by their position in each
step: the last dispatches of the run repeat the per-step GEMM sequence of --config (config 3:
forward, dW, dcol; config 5 adds the offset conv's GEMMs), and the mapping is accepted only if
every repetition has the same kernel at the same position.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

N_SIMD = 1024  # 256 CUs x 4 SIMDs (MI355X)
N_XCD = 8
PEAK_GHZ = 2.4  # MI355X peak engine clock (the 2.5 PF bf16 / 157.3 TF f32 MFMA spec clock)

# libdcn kernels -> bench.py scope (DCN_K_* class); first matching prefix wins
DCN_SCOPES = [
    ("dcn::fwd_fused_bf16", "gemm_fwd"),
    ("dcn::fwd_fused_f32", "gemm_fwd"),
    ("dcn::dw_stream_bf16", "gemm_dw"),
    ("dcn::dw_fused_bf16", "gemm_dw"),
    ("dcn::dcol_bf16", "gemm_dcol"),
    ("dcn::gemm_split", "gemm_split"),
    ("dcn::offset_conv_fwd", "offset_fwd"),
    ("dcn::offset_wgrad", "offset_bwd"),
    ("dcn::offset_dgrad", "offset_bwd"),
]
# per-step Cijk sequence by BASELINE config (dcn_api.cpp core_forward / core_backward order)
CIJK_CYCLE = {
    3: ["gemm_fwd", "gemm_dw", "gemm_dcol"],
    2: ["gemm_fwd"],
    5: ["offset_fwd", "gemm_fwd", "gemm_dw", "gemm_dcol", "offset_bwd", "offset_bwd"],
    4: [],
}
# kernels of the other forward schedules that bench.py --config 4 also times (fwd_paths: the
# no-column path): reported per kernel, kept out of the default step's scopes
NOT_DEFAULT = {4: ("dcn::dw_fused_bf16", "dcn::fwd_fused_bf16<false>")}
# exact MFMA counts of in-house kernels at config 4, for the counter's calibration:
# fwd_fused_bf16: 512 workgroups x 4 waves x 72 k-steps x 28 v_mfma_f32_16x16x32_bf16
CALIBRATION = {4: {"dcn::fwd_fused_bf16<true>": (512 * 4 * 72 * 28, 16)}}


def short(name):
    return name.replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0]


def load(d):
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not f:
        raise SystemExit(f"no counter_collection.csv under {d}")
    rows = defaultdict(dict)  # dispatch id -> {counter: value, name, t0, t1}
    for r in csv.DictReader(open(f[0])):
        did = int(r["Dispatch_Id"])
        e = rows[did]
        e["name"] = r["Kernel_Name"]
        e[r["Counter_Name"]] = e.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        if r.get("Start_Timestamp") and r.get("End_Timestamp"):
            e["t0"], e["t1"] = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    kt = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    if kt:  # durations from the kernel trace where it has the dispatch
        for r in csv.DictReader(open(kt[0])):
            did = int(r["Dispatch_Id"])
            if did in rows:
                rows[did]["t0"], rows[did]["t1"] = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    return [dict(rows[k], id=k) for k in sorted(rows)]


def cijk_scopes(disp, cycle):
    """Dispatch id -> scope for the Cijk dispatches of the repeating tail (see module doc)."""
    gem = [e for e in disp if e["name"].startswith("Cijk")]
    n = len(cycle)
    if not n or len(gem) < n:
        return {}, 0
    reps = []
    i = len(gem)
    while i - n >= 0:
        grp = gem[i - n:i]
        if reps and [short(e["name"]) for e in grp] != [short(e["name"]) for e in reps[0]]:
            break
        reps.append(grp)
        i -= n
    out = {}
    for grp in reps:
        for pos, e in enumerate(grp):
            out[e["id"]] = cycle[pos]
    return out, len(reps)


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    config = 3
    for a in sys.argv[1:]:
        if a.startswith("--config="):
            config = int(a.split("=", 1)[1])
    d, out = args[:2]
    disp = load(d)
    cmap, nrep = cijk_scopes(disp, CIJK_CYCLE.get(config, []))
    kern = defaultdict(lambda: defaultdict(float))
    scope = defaultdict(lambda: defaultdict(float))
    scope_k = defaultdict(set)
    for e in disp:
        nm = e["name"]
        if "SQ_VALU_MFMA_BUSY_CYCLES" not in e or "GRBM_GUI_ACTIVE" not in e:
            continue
        if nm.startswith("Cijk"):
            if e["id"] not in cmap:
                continue  # autotune candidates and warm-up launches
            sk = short(nm)
            sc = cmap[e["id"]]
            key = f"{sc}:{sk[:80]}"
        else:
            sk = short(nm)
            if not sk.startswith("dcn::"):
                continue
            sc = next((s for p, s in DCN_SCOPES if sk.startswith(p)), None)
            if sk.startswith(NOT_DEFAULT.get(config, ())):
                sc = None
            key = sk
        k = kern[key]
        k["launches"] += 1
        k["busy"] += e["SQ_VALU_MFMA_BUSY_CYCLES"]
        k["gui"] += e["GRBM_GUI_ACTIVE"]
        k["sq_busy"] += e.get("SQ_BUSY_CYCLES", 0.0)
        k["wave_cycles"] += e.get("SQ_WAVE_CYCLES", 0.0)
        if "t0" in e:
            k["ns"] += e["t1"] - e["t0"]
        if sc:
            s = scope[sc]
            s["busy"] += e["SQ_VALU_MFMA_BUSY_CYCLES"]
            s["cycles"] += e["GRBM_GUI_ACTIVE"] / N_XCD
            s["ns"] += e.get("t1", 0) - e.get("t0", 0)
            scope_k[sc].add(key)
    res_k = {}
    for key, k in sorted(kern.items(), key=lambda kv: -kv[1]["busy"]):
        n = k["launches"]
        cyc = k["gui"] / N_XCD / n
        r = {"launches": int(n), "mfma_busy_cycles": k["busy"] / n, "grbm_gui_active": k["gui"] / n,
             "cycles": cyc, "sq_busy_cycles": k["sq_busy"] / n, "sq_wave_cycles": k["wave_cycles"] / n,
             "mfma_busy": None,
             "mfma_busy_gui": round(k["busy"] / n / (N_SIMD * cyc), 4) if cyc else None}
        if k["ns"]:
            r["duration_ns"] = k["ns"] / n
            r["clock_ghz"] = round(cyc / (k["ns"] / n), 3)
            r["mfma_busy"] = round(k["busy"] / (N_SIMD * PEAK_GHZ * k["ns"]), 4)
        res_k[key] = r
    res_s = {}
    for sc, s in scope.items():
        res_s[sc] = {"kernels": sorted(scope_k[sc]),
                     "mfma_busy": round(s["busy"] / (N_SIMD * PEAK_GHZ * s["ns"]), 4)
                     if s["ns"] > 0 else None,
                     "mfma_busy_gui": round(s["busy"] / (N_SIMD * s["cycles"]), 4) if s["cycles"] else None,
                     "clock_ghz": round(s["cycles"] / s["ns"], 3) if s["ns"] > 0 else None,
                     "duration_ns": s["ns"]}
    calib = {}
    for nm, (n_mfma, cyc_per) in CALIBRATION.get(config, {}).items():
        if nm in res_k:
            calib[nm] = {"expected_busy_cycles": n_mfma * cyc_per,
                         "measured": res_k[nm]["mfma_busy_cycles"],
                         "ratio": round(res_k[nm]["mfma_busy_cycles"] / (n_mfma * cyc_per), 4)}
    doc = {"source": "tools/pmc_mfma.sh (rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES "
                     "SQ_WAVE_CYCLES GRBM_GUI_ACTIVE --kernel-trace) of bench.py "
                     f"--config {config} --steps 3 --warmup 2",
           "formula": "mfma_busy = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x 2.4 GHz x duration); "
                      "mfma_busy_gui = busy / (1024 x GRBM_GUI_ACTIVE / 8); scope = sums over its "
                      "kernels' dispatches",
           "config": config, "cijk_steps_attributed": nrep, "calibration": calib,
           "scopes": res_s, "kernels": res_k}
    with open(out, "w") as f:
        json.dump(doc, f, indent=1)
    for sc, v in sorted(res_s.items()):
        print(f"{sc:12s} mfma_busy {v['mfma_busy']}  clock {v['clock_ghz']} GHz  {v['kernels']}")
    for nm, v in calib.items():
        print("calibration", nm, v)


if __name__ == "__main__":
    main()
