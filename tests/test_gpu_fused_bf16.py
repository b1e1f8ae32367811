"""GPU parity of the bf16 fused forward (csrc/dcn_fused_bf16.hip): the
bilinear gather of deform_conv.py:47-54 fed from an LDS window of the channels-last x straight
into the B operand of bf16 MFMAs computing :76-80, the columns written only for a backward
that reuses them (DCN_FWD_FUSED) or never (DCN_FWD_FUSED_NOCOL).

* against the unfused schedule (K1 + hipBLASLt + bias, DCN_FWD_UNFUSED) on the same handle:
  out within one bf16 rounding of a different fp32 summation order; the columns the fused
  kernel stores bit for bit K1's, checked through the backward, whose ∂W GEMM reads them
  (DCN_BWD_COL_IN_WS): every gradient identical;
* DCN_FWD_FUSED_NOCOL (no column matrix anywhere in the step): out bit for bit the storing
  kernel's; its backward computes ∂W with the columns recomputed inside the MFMA kernel
  (dw_fused_bf16): ∂W within one bf16 rounding of the GEMM schedule's (another fp32 summation
  order) and against the oracle, every other gradient bit for bit;
* against the oracle (the bf16 tolerance of test_gpu_bf16);
* many samples outside the tile's LDS window (offset scale 3-8 px): the per-tile overflow
  area and, past its 48 entries, the in-line global corner reads;
* config 4 at full size: forward twice in one process, bit for bit.
"""
import ctypes

import numpy as np
import pytest

import dcn_oracle as O
import dcn_runtime as rt
from test_gpu_bf16 import Buf, _case, _device, assert_bf16_close

pytestmark = pytest.mark.gpu

CASES = [
    dict(seed=901, B=2, C=256, O_=256, H=28, W=28),                 # config 4 geometry
    dict(seed=902, B=2, C=64, O_=256, H=20, W=17, off_scale=2.0),   # ragged tiles (7x16)
    dict(seed=903, B=3, C=128, O_=512, H=24, W=24, s=(2, 2)),       # stride 2, 2 O tiles
    dict(seed=904, B=1, C=64, O_=256, H=9, W=40, k=(3, 2), p=(1, 0)),  # 6 taps, 3 tile cols
    dict(seed=905, B=2, C=192, O_=256, H=15, W=30, off_scale=3.0),  # overflow area in use
    dict(seed=906, B=2, C=64, O_=256, H=16, W=16, off_scale=8.0),   # past the overflow area
    dict(seed=907, B=2, C=64, O_=256, H=11, W=13, k=(1, 1), p=(0, 0)),  # 1 tap
]


def _run(h, c, path, pad=None):
    bits, v, s = c
    h.set_fwd_path(path)
    try:
        return _device(h, bits, s, pad=pad or (1, 1))
    finally:
        h.set_fwd_path(rt.DCN_FWD_AUTO)


def _pad(case):
    return case.get("p", (1, 1))


def _near(a, r, what):
    """One bf16 rounding of two fp32 sums that differ only in summation order."""
    d = np.abs(a.astype(np.float64) - r)
    rms = float(np.sqrt(np.mean(r.astype(np.float64) ** 2)))
    lim = 2.0 ** -7 * np.abs(r) + 2.0 ** -14 * rms
    assert np.all(d <= lim), f"{what}: {int((d > lim).sum())} elements past one bf16 ulp"


@pytest.mark.parametrize("case", CASES)
def test_fused_bf16_vs_unfused_and_oracle(gpu_handle, case):
    c = _case(**case)
    pad = _pad(case)
    out_f, off_f, g_f = _run(gpu_handle, c, rt.DCN_FWD_FUSED, pad)
    out_u, off_u, g_u = _run(gpu_handle, c, rt.DCN_FWD_UNFUSED, pad)
    np.testing.assert_array_equal(off_f, off_u)
    _near(out_f, out_u, f"fused vs unfused out {case}")
    # the stored columns are K1's bit for bit -> the whole backward is bitwise equal
    for k in g_u:
        np.testing.assert_array_equal(g_f[k], g_u[k], err_msg=f"∂{k} (columns differ) {case}")
    _, v, s = c
    ro, _, _ = O.forward(v["x"], v["w_off"], v["b_off"], v["w"], v["b"], s, pad, offsets=off_f)
    assert_bf16_close(out_f, ro, f"fused out vs oracle {case}")


@pytest.mark.parametrize("case", CASES)
def test_fused_bf16_nocol(gpu_handle, case):
    c = _case(**case)
    pad = _pad(case)
    out_f, _, _ = _run(gpu_handle, c, rt.DCN_FWD_FUSED, pad)
    out_n, off_n, g_n = _run(gpu_handle, c, rt.DCN_FWD_FUSED_NOCOL, pad)
    _, _, g_u = _run(gpu_handle, c, rt.DCN_FWD_UNFUSED, pad)
    np.testing.assert_array_equal(out_n.view(np.uint32), out_f.view(np.uint32))
    for k in g_u:
        if k == "weight":  # recomputed columns, another fp32 summation order
            _near(g_n[k], g_u[k], f"nocol ∂W vs GEMM {case}")
        else:
            np.testing.assert_array_equal(g_n[k], g_u[k], err_msg=f"nocol ∂{k}")
    _, v, s = c
    _, _, cache = O.forward(v["x"], v["w_off"], v["b_off"], v["w"], v["b"], s, pad,
                            offsets=off_n)
    rg = O.backward(cache, v["grad_out"])
    assert_bf16_close(g_n["weight"], rg["weight"], f"nocol ∂W vs oracle {case}")


def test_fused_bf16_config4_full_size_bitwise(gpu_handle):
    """BASELINE config 4 per GPU (B=64, C=O=256, 28x28): the fused forward twice in one
    process, bit for bit, and against the unfused schedule within one bf16 rounding."""
    c = _case(12, B=64, C=256, O_=256, H=28, W=28, off_scale=1.5)
    r1 = _run(gpu_handle, c, rt.DCN_FWD_FUSED)
    r2 = _run(gpu_handle, c, rt.DCN_FWD_FUSED)
    np.testing.assert_array_equal(r1[0].view(np.uint32), r2[0].view(np.uint32), err_msg="out")
    for k in r1[2]:
        np.testing.assert_array_equal(r1[2][k].view(np.uint32), r2[2][k].view(np.uint32),
                                      err_msg=k)
    ru = _run(gpu_handle, c, rt.DCN_FWD_UNFUSED)
    _near(r1[0], ru[0], "config 4 fused vs unfused out")
    for k in ru[2]:
        np.testing.assert_array_equal(r1[2][k], ru[2][k], err_msg=f"config 4 ∂{k}")


def test_fused_bf16_nocol_config4_full_size(gpu_handle):
    """BASELINE config 4 per GPU with no column matrix (fused forward, recomputed ∂W): twice
    in one process bit for bit, and against the column schedule (∂W within one bf16
    rounding, every other tensor bit for bit)."""
    c = _case(13, B=64, C=256, O_=256, H=28, W=28, off_scale=1.5)
    r1 = _run(gpu_handle, c, rt.DCN_FWD_FUSED_NOCOL)
    r2 = _run(gpu_handle, c, rt.DCN_FWD_FUSED_NOCOL)
    np.testing.assert_array_equal(r1[0].view(np.uint32), r2[0].view(np.uint32), err_msg="out")
    for k in r1[2]:
        np.testing.assert_array_equal(r1[2][k].view(np.uint32), r2[2][k].view(np.uint32),
                                      err_msg=k)
    ru = _run(gpu_handle, c, rt.DCN_FWD_UNFUSED)
    _near(r1[0], ru[0], "config 4 nocol vs unfused out")
    for k in ru[2]:
        if k == "weight":
            _near(r1[2][k], ru[2][k], "config 4 nocol ∂W")
        else:
            np.testing.assert_array_equal(r1[2][k], ru[2][k], err_msg=f"config 4 nocol ∂{k}")


def _upload_case(D, c):
    bits, _, s = c
    B, C, H, W = bits["x"].shape
    O_, _, kh, kw = bits["w"].shape
    J = bits["w_off"].shape[0]
    desc = rt.make_desc(B, C, H, W, O_, (kh, kw), s, (1, 1), dtype=rt.DCN_BF16)
    Ho, Wo = rt.out_shape(desc)
    p = {k: D.up(v) for k, v in bits.items()}
    p["out"], p["off"] = D.zeros(B * O_ * Ho * Wo * 2), D.zeros(B * J * Ho * Wo * 2)
    p["g"] = {k: D.zeros(v.nbytes) for k, v in bits.items() if k != "grad_out"}
    p["goff"] = D.zeros(B * J * Ho * Wo * 2)
    return desc, (B, O_, Ho, Wo), p


def _fwd(h, desc, p, ws, wsb, flags=0):
    vp = ctypes.c_void_p
    rt.check(h.lib.dcn_forward_ex(h.h, desc, vp(p["x"]), vp(p["w_off"]), vp(p["b_off"]),
                                  vp(p["w"]), vp(p["b"]), vp(p["out"]), vp(p["off"]), vp(ws),
                                  wsb, flags), "dcn_forward_ex")


def _bwd(h, desc, p, ws, wsb):
    vp = ctypes.c_void_p
    g = p["g"]
    rt.check(h.lib.dcn_backward(h.h, desc, vp(p["x"]), vp(p["off"]), vp(p["w_off"]), vp(p["w"]),
                                vp(p["grad_out"]), vp(g["x"]), vp(g["w"]), vp(g["b"]),
                                vp(g["w_off"]), vp(g["b_off"]), vp(p["goff"]), vp(ws), wsb,
                                rt.DCN_BWD_COL_IN_WS), "dcn_backward")


def _grads(D, c, p):
    bits = c[0]
    g = p["g"]
    return {"x": D.down(g["x"], bits["x"].shape), "weight": D.down(g["w"], bits["w"].shape),
            "bias": D.down(g["b"], bits["b"].shape),
            "offset_conv.weight": D.down(g["w_off"], bits["w_off"].shape),
            "offset_conv.bias": D.down(g["b_off"], bits["b_off"].shape)}


@pytest.mark.parametrize("path", [rt.DCN_FWD_FUSED_NOCOL, rt.DCN_FWD_AUTO])
def test_nocol_state_is_per_workspace(gpu_handle, path):
    """Several modules on one handle (a stack: all forwards, then all backwards), each with its
    own workspace, every backward with DCN_BWD_COL_IN_WS. Forwards without columns
    (DCN_FWD_FUSED_NOCOL on the handle, or DCN_FWD_NO_COLUMNS per call) are remembered per
    workspace, so every backward recomputes its columns instead of reading another step's;
    a column-storing forward in between on one of them makes that one read its columns again.
    Every module's gradients equal the unfused schedule's (∂W within one bf16 rounding where
    it is recomputed inside dw_fused_bf16, everything else bit for bit). deform_conv.py:41-80
    and its autodiff."""
    h = gpu_handle
    cases = [_case(930 + i, B=2, C=64, O_=256, H=28, W=28, off_scale=1.5) for i in range(3)]
    ref = [_run(h, c, rt.DCN_FWD_UNFUSED)[2] for c in cases]
    D = Buf(h)
    try:
        mods = [_upload_case(D, c) for c in cases]
        wsb = rt.workspace_bytes(mods[0][0], True)
        wss = [D.zeros(wsb) for _ in mods]
        h.set_fwd_path(path)
        flags = rt.DCN_FWD_NO_COLUMNS if path == rt.DCN_FWD_AUTO else 0
        for (desc, _, p), ws in zip(mods, wss):
            _fwd(h, desc, p, ws, wsb, flags)
        # module 1 runs a column-storing forward again (AUTO, no flag): its backward reads them
        h.set_fwd_path(rt.DCN_FWD_AUTO)
        _fwd(h, mods[1][0], mods[1][2], wss[1], wsb, 0)
        h.set_fwd_path(path)
        for (desc, _, p), ws in reversed(list(zip(mods, wss))):
            _bwd(h, desc, p, ws, wsb)
        for i, (c, (_, _, p)) in enumerate(zip(cases, mods)):
            got = _grads(D, c, p)
            for k in got:
                recomputed = k == "weight" and path == rt.DCN_FWD_FUSED_NOCOL and i != 1
                if recomputed:
                    _near(got[k], ref[i][k], f"module {i} ∂W (recomputed columns)")
                else:
                    np.testing.assert_array_equal(got[k], ref[i][k], err_msg=f"module {i} ∂{k}")
    finally:
        h.set_fwd_path(rt.DCN_FWD_AUTO)
        D.free()


def test_forward_no_columns_flag_small_workspace(gpu_handle):
    """dcn_forward_ex(DCN_FWD_NO_COLUMNS) in a workspace of dcn_workspace_bytes(d,
    DCN_WS_FORWARD_NO_COLUMNS) bytes (no column region: smaller by B·HW·K floats of the
    layout): out bit for bit the fused forward's, the handle's path untouched; a workspace
    one byte short is refused."""
    h = gpu_handle
    c = _case(940, B=2, C=128, O_=256, H=28, W=28)
    out_f, _, _ = _run(h, c, rt.DCN_FWD_FUSED)
    D = Buf(h)
    try:
        desc, oshape, p = _upload_case(D, c)
        full = rt.workspace_bytes(desc, False)
        small = rt.workspace_bytes(desc, rt.DCN_WS_FORWARD_NO_COLUMNS)
        B, C = c[0]["x"].shape[:2]
        assert full - small >= B * 28 * 28 * 9 * C * 4
        ws = D.zeros(small)
        h.set_fwd_path(rt.DCN_FWD_UNFUSED)
        _fwd(h, desc, p, ws, small, rt.DCN_FWD_NO_COLUMNS)
        assert h.get_fwd_path() == rt.DCN_FWD_UNFUSED
        out = D.down(p["out"], oshape)
        np.testing.assert_array_equal(out.view(np.uint32), out_f.view(np.uint32))
        vp = ctypes.c_void_p
        rc = h.lib.dcn_forward_ex(h.h, desc, vp(p["x"]), vp(p["w_off"]), vp(p["b_off"]),
                                  vp(p["w"]), vp(p["b"]), vp(p["out"]), vp(p["off"]), vp(ws),
                                  small - 1, rt.DCN_FWD_NO_COLUMNS)
        assert rc == -5  # DCN_ERR_WORKSPACE
    finally:
        h.set_fwd_path(rt.DCN_FWD_AUTO)
        D.free()


def test_column_record_stays_bounded(gpu_handle):
    """the handle's per-workspace column record must not grow with the number of
    distinct workspaces. 100 no-grad forwards (DCN_FWD_NO_COLUMNS) on fresh workspaces add
    nothing; 300 column-storing forwards on fresh workspaces keep at most 256 records (the
    oldest dropped). A backward with DCN_BWD_COL_IN_WS on a dropped workspace — whose column
    region later forwards have overwritten — recomputes the columns: every gradient bit for
    bit the unfused schedule's (deform_conv.py:41-80 and its autodiff)."""
    h = gpu_handle
    c = _case(950, B=1, C=64, O_=256, H=28, W=28, off_scale=1.5)
    ref = _run(h, c, rt.DCN_FWD_UNFUSED)[2]
    D = Buf(h)
    n = ctypes.c_int()

    def records():
        rt.check(h.lib.dcn_debug_col_ws_records(h.h, ctypes.byref(n)))
        return n.value

    try:
        desc, _, p = _upload_case(D, c)
        wsb = rt.workspace_bytes(desc, True)
        big = D.zeros(wsb + 400 * 256)  # workspace i at big + 256·i: all distinct addresses
        ws = lambda i: big + 256 * i
        r0 = records()
        for i in range(100):
            _fwd(h, desc, p, ws(i), wsb, rt.DCN_FWD_NO_COLUMNS)
        assert records() <= r0  # (a recorded address may recur among the fresh ones)
        for i in range(300):
            _fwd(h, desc, p, ws(100 + i), wsb, 0)
        assert records() <= 256
        _bwd(h, desc, p, ws(100), wsb)  # dropped long ago, its columns overwritten
        got = _grads(D, c, p)
        for k in got:
            np.testing.assert_array_equal(got[k], ref[k], err_msg=f"∂{k} on a dropped workspace")
        _fwd(h, desc, p, ws(399), wsb, 0)  # the newest record: its columns are read
        _bwd(h, desc, p, ws(399), wsb)
        got = _grads(D, c, p)
        for k in got:
            np.testing.assert_array_equal(got[k], ref[k], err_msg=f"∂{k} on a recorded workspace")
    finally:
        D.free()
