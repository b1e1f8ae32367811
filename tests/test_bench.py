"""CPU: bench.py's measurement arithmetic (no GPU). The algorithmic bytes and FLOPs the
roofline fractions divide by must be SURVEY §8(d)'s figures, and every BASELINE config must
be a bench workload."""
import importlib.util
import os

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def bench():
    spec = importlib.util.spec_from_file_location("bench", os.path.join(ROOT, "bench.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def test_k1_algorithmic_bytes_match_survey(bench):
    # config 3 K1 = 2,069,659,648 B (1,145.8 B/sample); config 4 bf16 with
    # bf16 offsets = 258,707,456 B
    assert bench.k1_bytes(64, 256, 56, 56, 9, 56, 56) == 2_069_659_648
    assert bench.k1_bytes(64, 256, 28, 28, 9, 28, 28, elem=2) == 258_707_456
    assert round(bench.k1_bytes(64, 256, 56, 56, 9, 56, 56) / (64 * 56 * 56 * 9), 1) == 1145.8


def test_other_rooflines_use_survey_work(bench):
    km = {"gemm_fwd": 1.5, "gemm_dw": 1.5, "gemm_dcol": 1.5, "col2im": 0.5}
    r = {e["kernel"].split(" ")[0]: e for e in
         bench.other_rooflines(km, 64, 256, 256, 56, 56, 9, 56, 56, 18, False, False)}
    # 2·M·K·O = 236,760,072,192 FLOP per GEMM at config 3
    assert r["gemm_fwd"]["algorithmic_flop"] == 236_760_072_192
    assert r["gemm_fwd"]["peak"] == 157.3 and r["gemm_fwd"]["unit"] == "TFLOP/s"
    assert abs(r["gemm_fwd"]["achieved"] - 236.76 / 1.5) < 0.1
    # K5 = 4·(M·K + 2·B·C·Hi·Wi + 2·B·2N·Ho·Wo) = 2,289,631,232 B
    assert r["col2im"]["algorithmic_bytes"] == 2_289_631_232
    assert r["col2im"]["bound"] == "hbm"
    # forward-only configs report the forward GEMM alone; bf16 prices against the bf16 peak
    fo = bench.other_rooflines(km, 8, 64, 128, 56, 56, 9, 56, 56, 18, False, True)
    assert [e["kernel"] for e in fo] == ["gemm_fwd"]
    b16 = bench.other_rooflines(km, 64, 256, 256, 28, 28, 9, 28, 28, 18, True, False)
    assert all(e["peak"] == 2500.0 for e in b16 if e["bound"] == "mfma")


def test_every_baseline_config_is_a_workload(bench):
    # BASELINE.json configs[0..4] = configs 1..5
    assert sorted(bench.CONFIGS) == [1, 2, 3, 4, 5]
    c3 = bench.CONFIGS[3]
    assert (c3["B"], c3["C"], c3["O"], c3["H"], c3["W"], c3["k"], c3["dtype"]) == \
        (64, 256, 256, 56, 56, 3, "f32")
    assert bench.CONFIGS[4]["dtype"] == "bf16" and bench.CONFIGS[2].get("fwd_only")
    c5 = bench.CONFIGS[5]
    assert (c5["s"], c5["dil"], c5["G"]) == (2, 2, 4)


def _run_bench(*argv, env=None, timeout=180):
    import json
    import subprocess
    import sys
    e = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        e.pop(k, None)
    e.update(env or {})
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *argv], env=e,
                       capture_output=True, text=True, timeout=timeout)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    return r.returncode, (json.loads(lines[-1]) if lines else None), r.stderr


@pytest.mark.parametrize("n", [2, 3])
def test_gpus_flag_spawns_that_many_ranks(n):
    """`bench.py --gpus N` with no external launcher starts N ranks itself (the driver may
    run it that way); --dry joins them in a gloo group without touching a GPU."""
    rc, line, err = _run_bench("--gpus", str(n), "--dry")
    assert rc == 0, err
    assert line["n_gpus"] == n and line["rank_id_sum"] == n * (n - 1) // 2


def test_world_size_mismatch_fails():
    rc, line, _ = _run_bench("--gpus", "2", "--dry",
                             env={"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert rc != 0 and line is None


def test_host_cpus_reports_model_and_count(bench):
    threads, info = bench.host_cpus()
    assert 1 <= threads <= info["host_threads"]
    assert threads <= info["affinity_threads"]
    assert "cpu_model" in info


def test_shard_sizes_split_a_fixed_global_batch(bench):
    """SURVEY §8(e) strong scaling: the fixed global batch of 512 over 1/2/4/8 GPUs."""
    for n, want in ((1, [512]), (2, [256] * 2), (4, [128] * 4), (8, [64] * 8)):
        assert bench.shard_sizes(512, n) == want
    assert bench.shard_sizes(10, 4) == [3, 3, 2, 2]  # ragged: the first ranks take one more
    with pytest.raises(ValueError):
        bench.shard_sizes(3, 4)


@pytest.mark.parametrize("n", [1, 2, 4, 8])
def test_dry_strong_scaling_shards_per_rank(n):
    """`bench.py --gpus N --global-batch 512 --dry`: every rank computes its own shard and
    rank 0 reports what the ranks gathered (gloo on CPU): 512 images in all, 512/N each."""
    rc, line, err = _run_bench("--gpus", str(n), "--global-batch", "512", "--dry", timeout=300)
    assert rc == 0, err
    assert line["scaling"] == "strong" and line["n_gpus"] == n
    assert line["shards"] == [512 // n] * n and line["global_batch"] == 512


def test_dry_weak_scaling_shards_per_rank():
    rc, line, err = _run_bench("--gpus", "2", "--dry")
    assert rc == 0, err
    assert line["scaling"] == "weak" and line["shards"] == [64, 64]


def test_config4_leg_is_wired(bench):
    """The default config-3 run times BASELINE config 4 beside the headline (VERDICT r03 next
    item 2): bf16, 64 images per GPU, C=O=256, 28x28, fwd+bwd, through the same timed() /
    warmup / steps, reported under `config4` with its kernel times, the dominant kernel's
    roofline (the fused forward against the bf16 MFMA peak when AUTO runs it, K1 bf16 against
    HBM otherwise) and the forward-schedule split. Stubbed device: only the wiring runs."""
    import argparse
    import sys
    sys.path.insert(0, os.path.join(ROOT, "jittor-dcn_amd"))
    torch = pytest.importorskip("torch")
    import dcn_dp
    import dcn_runtime as rt
    c4 = bench.CONFIGS[4]
    assert (c4["B"], c4["C"], c4["O"], c4["H"], c4["W"], c4["k"], c4["dtype"]) == \
        (64, 256, 256, 28, 28, 3, "bf16")
    wl = bench.Workload(c4, rt, torch, torch.device("cpu"), dcn_dp, seed=4321)
    assert wl.w.dtype == torch.bfloat16 and wl.desc(64).dtype == rt.DCN_BF16
    calls = {}

    def make_step(w, nb, seed):
        calls["make_step"] = (w.cfg is c4, nb)
        return (lambda: calls.__setitem__("steps", calls.get("steps", 0) + 1)), ()

    def timed(step, steps):
        calls["timed"] = steps
        return 0.7e-3 * steps

    for km, kind in (({"gemm_fwd": 0.14, "gemm_dw": 0.12, "gemm_dcol": 0.1, "col2im": 0.11},
                      "mfma"),
                     ({"im2col": 0.07, "gemm_fwd": 0.08, "gemm_dw": 0.12}, "hbm")):
        args = argparse.Namespace(warmup=2, steps=5, fwd_path=0, exchange=False)
        res = bench.config4_leg(args, 1, 0, wl, rt, make_step, timed, lambda s, n: km,
                                lambda s, w, n: {"fused": 0.7}, lambda: None)
        assert calls["make_step"] == (True, 64) and calls["timed"] == 5
        assert res["dtype"] == "bf16" and res["unit"] == "Gsamples/s"
        assert res["workload"].startswith("config4: B=64/GPU C=256->O=256 28x28 k3")
        assert abs(res["ms_per_step"] - 0.7) < 1e-9
        # 64·28·28·9 samples per 0.7 ms
        assert abs(res["value"] - 64 * 28 * 28 * 9 / 0.7e-3 / 1e9) < 1e-4
        assert res["kernel_ms"] is km and res["fwd_paths_ms_per_step"] == {"fused": 0.7}
        assert res["roofline"]["bound"] == kind
        for key in ("achieved", "peak", "unit", "frac"):
            assert key in res["roofline"]
    # at N > 1 the leg reports the whole job (every rank's 64 images), no schedule split
    res = bench.config4_leg(argparse.Namespace(warmup=1, steps=2, fwd_path=0, exchange=False),
                            8, 0, wl, rt, make_step, timed, lambda s, n: {"gemm_fwd": 0.14},
                            lambda s, w, n: {"x": 1}, lambda: None)
    assert res["n_gpus"] == 8 and res["global_batch"] == 512 and res["fwd_paths_ms_per_step"] is None
    assert "all-reduce" in res["workload"]


def test_scope_rooflines_use_survey_work(bench):
    """Every timed scope against its bound, the longest first (the dominant kernel)."""
    c3 = bench.CONFIGS[3]
    km = {"gemm_fwd": 1.6, "im2col": 0.4, "col2im": 0.52, "offset_fwd": 0.2, "offset_bwd": 0.4,
          "bias_fwd": 0.06, "unknown_scope": 9.0}
    r = bench.scope_rooflines(km, c3, 64, 56, 56)
    assert [e["kernel"] for e in r] == ["gemm_fwd", "col2im", "im2col", "offset_bwd",
                                        "offset_fwd", "bias_fwd"]
    by = {e["kernel"]: e for e in r}
    assert by["im2col"]["algorithmic_bytes"] == 2_069_659_648
    assert by["col2im"]["algorithmic_bytes"] == 2_289_631_232
    assert by["gemm_fwd"]["algorithmic_flop"] == 236_760_072_192
    # offset conv: 2·M·K·2N = 16.65 GFLOP at config 3, its backward twice that
    assert abs(by["offset_fwd"]["algorithmic_flop"] - 16.65e9) < 0.01e9
    assert by["offset_bwd"]["algorithmic_flop"] == 2 * by["offset_fwd"]["algorithmic_flop"]
    assert by["gemm_fwd"]["peak"] == 157.3 and by["im2col"]["peak"] == bench.HBM_PEAK_GBS
    c5 = bench.CONFIGS[5]  # 4 deform groups: J = 72 offset channels
    r5 = {e["kernel"]: e for e in bench.scope_rooflines({"im2col": 0.1}, c5, 64, 6, 6)}
    assert r5["im2col"]["algorithmic_bytes"] == 4 * (64 * 512 * 14 * 14 + 64 * 72 * 36
                                                      + 64 * 36 * 9 * 512)


@pytest.mark.parametrize("num", [2, 5])
def test_extra_config_legs_are_wired(bench, num):
    """BASELINE configs 2 (fp32 forward only, vs CPU) and 5 (the
    DCNv1 option set) are timed in the default N=1 run through the same timed() / warmup /
    steps and reported under `config2` / `config5` with kernel times, the dominant scope's
    roofline and, for config 2, its own CPU baseline. Stubbed device: only the wiring runs."""
    import argparse
    import sys
    sys.path.insert(0, os.path.join(ROOT, "jittor-dcn_amd"))
    torch = pytest.importorskip("torch")
    import dcn_dp
    import dcn_runtime as rt
    cfg = bench.CONFIGS[num]
    wl = bench.Workload(cfg, rt, torch, torch.device("cpu"), dcn_dp, seed=6000 + num)
    assert wl.desc(cfg["B"]).dtype == rt.DCN_F32
    calls = {}

    def make_step(w, nb, seed):
        calls["make_step"] = (w.cfg is cfg, nb)
        return (lambda: None), ()

    def timed(step, steps):
        calls["timed"] = steps
        return 0.1e-3 * steps

    km = ({"offset_fwd": 0.01, "im2col": 0.02, "gemm_fwd": 0.04, "bias_fwd": 0.01} if num == 2
          else {"gemm_fwd": 0.08, "gemm_dw": 0.09, "gemm_dcol": 0.08, "col2im": 0.05})
    cpu = {"value": 0.005, "unit": "Gsamples/s"}
    args = argparse.Namespace(warmup=2, steps=5)
    res = bench.extra_config_leg(num, args, wl, rt, make_step, timed, lambda s, n: km,
                                 lambda: None, cpu, lambda s, n: 0.05)
    assert res["graph_ms_per_step"] == 0.05
    assert calls["make_step"] == (True, cfg["B"]) and calls["timed"] == 5
    Ho, Wo = rt.out_shape(wl.desc(cfg["B"]))
    assert (Ho, Wo) == ((56, 56) if num == 2 else (6, 6))
    assert res["samples_per_step"] == cfg["B"] * Ho * Wo * 9
    assert abs(res["value"] - res["samples_per_step"] / 0.1e-3 / 1e9) < 1e-4
    assert res["workload"].startswith(f"config{num}: B={cfg['B']}/GPU")
    assert ("fwd only" in res["workload"]) == (num == 2)
    assert res["roofline"]["kernel"] == max(km, key=km.get)
    assert len(res["rooflines_other"]) == len(km) - 1
    assert res["cpu_baseline"] is cpu and res["gpu_over_cpu"] > 1


def test_config5_cpu_baseline_runs_the_c_port(bench):
    """VERDICT r05 missing 5: config 5 (dilation 2, 4 deform groups) has a CPU baseline, the
    fp32 C/OpenMP restatement (oracle/dcn_ref.c), which supports both; a bounded sample."""
    r = bench.cpu_baseline(bench.CONFIGS[5], budget_s=0.05, threads=2, name="config5")
    assert r["kind"] == "port" and r["unit"] == "Gsamples/s" and r["value"] > 0
    assert r["cores"] == 2 and "config5" in r["sample"] and "1x512x14x14" in r["sample"]


def test_mfma_busy_is_wired(bench, tmp_path, monkeypatch):
    """every MFMA-bound roofline carries the counter-measured MFMA
    utilisation (`mfma_busy`, `busy_source`) from the newest committed
    profiles/r*_mfma_busy_config{N}.json; HBM-bound entries are left alone."""
    import json
    prof = tmp_path / "profiles"
    prof.mkdir()
    doc = {"scopes": {"gemm_fwd": {"mfma_busy": 0.81, "clock_ghz": 2.05},
                      "offset_bwd": {"mfma_busy": 0.5, "clock_ghz": 2.1}}}
    (prof / "r99_mfma_busy_config3.json").write_text(json.dumps(doc))
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    km = {"gemm_fwd": 1.6, "gemm_dw": 1.6, "col2im": 0.5, "offset_bwd": 0.4}
    ent = bench.other_rooflines(km, 64, 256, 256, 56, 56, 9, 56, 56, 18, False, False)
    ent += [e for e in bench.scope_rooflines(km, bench.CONFIGS[3], 64, 56, 56)
            if e["kernel"] == "offset_bwd"]
    by = {e["kernel"].split(" ")[0]: e for e in bench.annotate_busy(ent, 3)}
    assert by["gemm_fwd"]["mfma_busy"] == 0.81 and by["gemm_fwd"]["busy_clock_ghz"] == 2.05
    assert by["gemm_fwd"]["busy_source"] == "profiles/r99_mfma_busy_config3.json:gemm_fwd"
    assert by["offset_bwd"]["mfma_busy"] == 0.5
    assert by["gemm_dw"]["mfma_busy"] is None and by["gemm_dw"]["busy_source"] is None
    assert "mfma_busy" not in by["col2im"]  # HBM-bound
    f = bench.annotate_busy([bench.fused_roofline({"gemm_fwd": 0.1}, 64, 28, 28, 9, 256, 256)], 3)
    assert f[0]["mfma_busy"] == 0.81  # the fused forward is the gemm_fwd scope
