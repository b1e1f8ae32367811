"""CPU: the C-ABI boundary — libdcn.so loads, exports every symbol include/dcn.h
declares, the ctypes prototypes cover the header, and the shape/validation
entry points behave without a device. No compute calls (no GPU here)."""
import ctypes
import os
import re
import subprocess

import pytest

import dcn_runtime as rt
from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "dcn.h")


def header_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:int|const char\*)\s+(dcn_\w+)\s*\(", src, flags=re.M)))


def test_library_exists_and_loads():
    assert os.path.exists(rt.LIB_PATH), "build libdcn.so first (__graft_entry__.build())"
    rt.load()


def test_every_header_symbol_is_exported():
    funcs = header_functions()
    assert len(funcs) >= 25
    out = subprocess.run(["nm", "-D", "--defined-only", rt.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    exported = set(re.findall(r"\bT (dcn_\w+)", out))
    missing = [f for f in funcs if f not in exported]
    assert not missing, f"declared in dcn.h but not exported: {missing}"


def test_ctypes_prototypes_cover_header():
    funcs = header_functions()
    assert sorted(rt.SIGNATURES) == funcs


def test_library_links_no_torch():
    out = subprocess.run(["ldd", rt.LIB_PATH], capture_output=True, text=True).stdout
    assert "torch" not in out and "libc10" not in out
    assert "librocblas" in out and "libamdhip64" in out


def test_desc_layout_matches_header():
    # dcn_desc = 16 ints
    assert ctypes.sizeof(rt.Desc) == 16 * 4


def desc(**kw):
    base = dict(B=2, C=4, H=9, W=11, O=3, kernel_size=(3, 3), stride=(1, 1), padding=(1, 1))
    base.update(kw)
    return rt.make_desc(**base)


def test_out_shape_and_workspace():
    assert rt.out_shape(desc()) == (9, 11)
    assert rt.out_shape(desc(stride=(2, 2))) == (5, 6)
    assert rt.out_shape(desc(H=14, W=14, stride=(2, 2), dilation=(2, 2))) == (6, 6)
    d = desc()
    fwd = rt.workspace_bytes(d, False)
    bwd = rt.workspace_bytes(d, True)
    K, HW = 9 * 4, 9 * 11
    assert fwd >= 2 * K * HW * 4
    assert bwd > fwd


@pytest.mark.parametrize("bad,msg", [
    (dict(B=0), "positive"),
    (dict(stride=(0, 1)), "positive"),
    (dict(H=2, W=2, padding=(0, 0)), "empty output"),
    (dict(H=3, W=8, padding=(0, 1)), "divides"),        # H_out == 1 (deform_conv.py:38)
    (dict(deform_groups=3), "divisible"),
    (dict(dtype=7), "unknown dtype"),
    (dict(dtype=rt.DCN_BF16, C=6), "DCN_BF16 needs"),      # C % 4 != 0
    (dict(dtype=rt.DCN_BF16, C=512), "DCN_BF16 needs"),    # C > 256
])
def test_invalid_descriptors_are_rejected(bad, msg):
    with pytest.raises(RuntimeError, match=msg):
        rt.out_shape(desc(**bad))


def test_no_device_fails_loudly():
    if rt.device_count() > 0:
        pytest.skip("a HIP device is visible")
    with pytest.raises(RuntimeError, match="dcn_create"):
        rt.Handle(0)
    assert rt.last_error() != ""


@pytest.mark.parametrize("shape", [dict(C=256, O=256, H=28, W=28), dict(C=64, O=128, H=13, W=17),
                                   dict(C=32, O=32, H=9, W=11, stride=(2, 2))])
def test_dw_partials_fit_the_workspace_layout(shape):
    """every ∂W path writes its partial planes into the workspace's
    `parts` region before the fixed-order sum. For every batch size 1..64, fp32 and bf16, each
    path's plane count (from the functions the backward itself uses) must fit what the
    dcn_forward + dcn_backward layout holds. Host only: no device call."""
    import ctypes
    L = rt.load()
    planes, cap = (ctypes.c_int * 4)(), ctypes.c_int()
    for dt in (rt.DCN_F32, rt.DCN_BF16):
        seen = set()
        for B in range(1, 65):
            d = desc(B=B, dtype=dt, **shape)
            rt.check(L.dcn_debug_dw_parts(ctypes.byref(d), planes, 4, ctypes.byref(cap)))
            n = list(planes)
            assert n[0] == B  # one plane per image
            assert max(n) <= cap.value, (dt, B, n, cap.value)
            seen.add(tuple(v > 0 for v in n))
        if dt == rt.DCN_BF16 and shape["C"] == 256:
            # the grouped GEMM (B % 16 == 0, B > 16), the recomputed-column kernel and the
            # streaming kernel (O == 256) apply
            assert (True, True, True, True) in seen
