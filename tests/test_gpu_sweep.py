"""GPU parity over a seeded sweep of random geometries (fp32, through the C-ABI device API).

Each case draws batch, channels, image size, kernel (1..3 x 1..3), stride (1..2), padding
(0..kernel-1), bias on/off and an offset scale from a fixed seed, skips the geometries the
reference itself cannot run (Ho or Wo == 1 divides by zero), and checks forward
and every gradient against the oracle at the north-star tolerance (conftest). Channel counts
cover every K1 / K5 instantiation: C % 4 != 0 (scalar lanes), C <= 32 / 64 / 128 windows,
C = 256 whole rows and C > 256 (lane-map loop). A second pass runs the same geometries
through the fused forward wherever it applies (C % 32 == 0, O % 128 == 0).
"""
import numpy as np
import pytest

import dcn_oracle as O
import dcn_runtime as rt
from test_gpu_parity import _check, _device_fwd_bwd, _oracle, _rand_case

pytestmark = pytest.mark.gpu

_CHANNELS = (3, 4, 12, 32, 64, 96, 128, 256, 288)


def _geometry(i):
    rng = np.random.default_rng(1000 + i)
    while True:
        kh, kw = int(rng.integers(1, 4)), int(rng.integers(1, 4))
        sh, sw = int(rng.integers(1, 3)), int(rng.integers(1, 3))
        ph, pw = int(rng.integers(0, kh)), int(rng.integers(0, kw))
        H, W = int(rng.integers(5, 24)), int(rng.integers(5, 24))
        Ho, Wo = O.out_size(H, W, kh, kw, sh, sw, ph, pw)
        if Ho >= 2 and Wo >= 2:
            break
    C = _CHANNELS[i % len(_CHANNELS)]
    O_ = int(rng.choice([5, 16, 128, 256]))
    return dict(seed=2000 + i, B=int(rng.integers(1, 4)), C=C, O_=O_, H=H, W=W, k=(kh, kw),
                s=(sh, sw), p=(ph, pw), off_scale=float(rng.choice([0.5, 1.0, 3.0])),
                bias=bool(rng.integers(0, 2)))


CASES = [_geometry(i) for i in range(18)]


@pytest.mark.parametrize("case", CASES, ids=[f"g{i}" for i in range(len(CASES))])
def test_random_geometry_vs_oracle(gpu_handle, case):
    c = _rand_case(**case)
    out, off, g = _device_fwd_bwd(gpu_handle, c)
    ro, roff, rg = _oracle(c, off)
    _check(out, off, g, ro, roff, rg, c["b"] is not None, str(case))


FUSED = [c for c in CASES if c["C"] % 32 == 0 and c["O_"] % 128 == 0 and c["k"][0] * c["k"][1] <= 9]


@pytest.mark.parametrize("case", FUSED, ids=[f"f{i}" for i in range(len(FUSED))])
def test_random_geometry_fused_forward(gpu_handle, case):
    c = _rand_case(**case)
    gpu_handle.set_fwd_path(rt.DCN_FWD_FUSED)
    try:
        out, off, g = _device_fwd_bwd(gpu_handle, c)
    finally:
        gpu_handle.set_fwd_path(rt.DCN_FWD_AUTO)
    ro, roff, rg = _oracle(c, off)
    _check(out, off, g, ro, roff, rg, c["b"] is not None, f"fused {case}")
