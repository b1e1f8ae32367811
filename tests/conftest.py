"""Shared pytest setup: marker registration, import paths, golden-fixture loader."""
from __future__ import annotations

import glob
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "jittor-dcn_amd")
for p in (ROOT, PKG, os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN_DIR = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device); run with -m gpu")


def golden_names():
    return sorted(os.path.splitext(os.path.basename(p))[0]
                  for p in glob.glob(os.path.join(GOLDEN_DIR, "*.npz")))


def load_golden(name):
    with np.load(os.path.join(GOLDEN_DIR, name + ".npz"), allow_pickle=False) as z:
        d = {k: z[k] for k in z.files}
    d["stride"] = tuple(int(v) for v in d["stride"])
    d["padding"] = tuple(int(v) for v in d["padding"])
    d["kernel"] = tuple(int(v) for v in d["kernel"])
    d.setdefault("b", None)
    return d


def assert_close(actual, ref, atol=1e-4, rtol=1e-4, what=""):
    """North-star tolerance: |Δ| <= 1e-4 + 1e-4·|ref| elementwise."""
    a = np.asarray(actual, np.float64)
    r = np.asarray(ref, np.float64)
    assert a.shape == r.shape, f"{what}: shape {a.shape} vs {r.shape}"
    bad = np.abs(a - r) > atol + rtol * np.abs(r)
    if bad.any():
        i = np.unravel_index(np.argmax(np.abs(a - r) - rtol * np.abs(r)), a.shape)
        raise AssertionError(f"{what}: {bad.sum()} / {a.size} elements out of tolerance; worst at "
                             f"{i}: got {a[i]!r} want {r[i]!r}")


def assert_close_reduction(actual, ref, tol=1e-4, what=""):
    """M-reductions (∂W, ∂b, ∂W_off, ∂b_off): max|Δ| / max|ref| <= 1e-4."""
    a = np.asarray(actual, np.float64)
    r = np.asarray(ref, np.float64)
    assert a.shape == r.shape, f"{what}: shape {a.shape} vs {r.shape}"
    scale = max(np.max(np.abs(r)), 1e-30)
    err = np.max(np.abs(a - r)) / scale
    assert err <= tol, f"{what}: max|Δ|/max|ref| = {err:.3e} > {tol:.0e}"


@pytest.fixture(scope="session")
def gpu_handle():
    import dcn_runtime as rt
    if rt.device_count() < 1:
        pytest.fail("no HIP device visible: -m gpu tests need an MI355X")
    return rt.Handle(0)
