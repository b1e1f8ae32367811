"""ctypes binding of libdcn.so (include/dcn.h) — the product's only path to the GPU.

The reference is a Jittor/NumPy code base (deform_conv.py, train.py), so the
operator is exposed as a plain C-ABI shared library bound with ctypes; there is
no torch extension and no CPU fallback: if the library or a HIP device is
missing every compute call raises RuntimeError.
"""
from __future__ import annotations

import ctypes
import os
import sys
import threading

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("DCN_LIB", os.path.join(HERE, "lib", "libdcn.so"))

ABI_VERSION = 5  # include/dcn.h DCN_ABI_VERSION
HOST_REUSE_FWD = 2  # include/dcn.h DCN_HOST_REUSE_FWD
DCN_F32, DCN_BF16 = 0, 1
DCN_BWD_COL_IN_WS = 1
DCN_FWD_NO_COLUMNS = 1  # dcn_forward_ex flag
DCN_WS_FORWARD_NO_COLUMNS = 2  # dcn_workspace_bytes(with_backward=2)
DCN_FWD_AUTO, DCN_FWD_UNFUSED, DCN_FWD_FUSED, DCN_FWD_FUSED_NOCOL = 0, 1, 2, 3
DCN_MATH_F32, DCN_MATH_F32_BF16X3, DCN_MATH_F32_BF16X6, DCN_MATH_F32_BF16X9 = 0, 3, 6, 9
KERNEL_IDS = {
    "offset_fwd": 0, "im2col": 1, "gemm_fwd": 2, "bias_fwd": 3, "bwd_bias": 4,
    "gemm_dw": 5, "gemm_dcol": 6, "col2im": 7, "offset_bwd": 8, "xpose": 9,
}


class Desc(ctypes.Structure):
    """dcn_desc (include/dcn.h)."""
    _fields_ = [(n, ctypes.c_int) for n in
                ("B", "C", "H", "W", "O", "kh", "kw", "sh", "sw", "ph", "pw", "dil_h", "dil_w",
                 "deform_groups", "dtype", "has_bias")]


class RoiDesc(ctypes.Structure):
    """dcn_roi_desc (include/dcn.h): DeformRoIPool / DeformPSRoIPool geometry."""
    _fields_ = [(n, ctypes.c_int) for n in ("B", "C", "H", "W", "R", "ph", "pw", "part_h",
                                            "part_w")] + \
               [("spatial_scale", ctypes.c_float), ("trans_std", ctypes.c_float),
                ("ps", ctypes.c_int), ("no_trans", ctypes.c_int)]


_vp = ctypes.c_void_p
_ip = ctypes.POINTER(ctypes.c_int)
_dp = ctypes.POINTER(Desc)
_sz = ctypes.c_size_t

# name -> argtypes (restype int unless listed in _RESTYPES). Mirrors include/dcn.h.
SIGNATURES = {
    "dcn_abi_version": [],
    "dcn_last_error": [],
    "dcn_device_count": [_ip],
    "dcn_create": [ctypes.c_int, ctypes.POINTER(_vp)],
    "dcn_destroy": [_vp],
    "dcn_set_stream": [_vp, _vp],
    "dcn_use_own_stream": [_vp],
    "dcn_get_stream": [_vp, ctypes.POINTER(_vp)],
    "dcn_synchronize": [_vp],
    "dcn_malloc": [_vp, _sz, ctypes.POINTER(_vp)],
    "dcn_free": [_vp, _vp],
    "dcn_host_alloc": [_vp, _sz, ctypes.POINTER(_vp)],
    "dcn_host_free": [_vp],
    "dcn_memcpy_h2d": [_vp, _vp, _vp, _sz],
    "dcn_memcpy_d2h": [_vp, _vp, _vp, _sz],
    "dcn_memset_zero": [_vp, _vp, _sz],
    "dcn_out_shape": [_dp, _ip, _ip],
    "dcn_workspace_bytes": [_dp, ctypes.c_int, ctypes.POINTER(_sz)],
    "dcn_offset_conv_fwd": [_vp, _dp, _vp, _vp, _vp, _vp],
    "dcn_offset_conv_bwd": [_vp, _dp, _vp, _vp, _vp, _vp, _vp, _vp],
    "dcn_im2col_fwd": [_vp, _dp, _vp, _vp, _vp, ctypes.c_int, ctypes.c_int],
    "dcn_col2im_coord_bwd": [_vp, _dp, _vp, _vp, _vp, _vp, _vp, ctypes.c_int, ctypes.c_int],
    "dcn_forward": [_vp, _dp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _sz],
    "dcn_forward_ex": [_vp, _dp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _sz, ctypes.c_int],
    "dcn_backward": [_vp, _dp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _sz,
                     ctypes.c_int],
    "dcn_forward_host": [_vp, _dp, _vp, _vp, _vp, _vp, _vp, _vp, _vp],
    "dcn_backward_host": [_vp, _dp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp],
    "dcn_backward_host_ex": [_vp, _dp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp,
                             ctypes.c_int],
    "dcn_host_state_create": [_vp, ctypes.POINTER(_vp)],
    "dcn_host_state_destroy": [_vp],
    "dcn_host_state_set_chunks": [_vp, ctypes.c_int],
    "dcn_forward_host_s": [_vp, _dp, _vp, _vp, _vp, _vp, _vp, _vp, _vp],
    "dcn_backward_host_s": [_vp, _dp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp,
                            ctypes.c_int],
    "dcn_prof_enable": [_vp, ctypes.c_int],
    "dcn_prof_read": [_vp, ctypes.c_int, ctypes.POINTER(ctypes.c_double), _ip],
    "dcn_prof_reset": [_vp],
    "dcn_comm_get_unique_id": [_vp],
    "dcn_comm_init": [_vp, ctypes.c_int, ctypes.c_int, _vp, ctypes.POINTER(_vp)],
    "dcn_comm_destroy": [_vp],
    "dcn_allreduce_grads": [_vp, _vp, _vp, _sz, ctypes.c_int],
    "dcn_set_comm": [_vp, _vp],
    "dcn_set_grad_stream": [_vp, _vp],
    "dcn_debug_force_generic": [ctypes.c_int],
    "dcn_set_math": [_vp, ctypes.c_int],
    "dcn_get_math": [_vp, _ip],
    "dcn_set_fwd_path": [_vp, ctypes.c_int],
    "dcn_get_fwd_path": [_vp, _ip],
    "dcn_debug_fused_workgroups": [ctypes.c_int],
    "dcn_debug_dw_parts": [_dp, _ip, ctypes.c_int, _ip],
    "dcn_debug_bins_chunked": [ctypes.c_int],
    "dcn_debug_offset_gemm": [ctypes.c_int],
    "dcn_debug_col_ws_records": [_vp, _ip],
    "dcn_debug_gemm": [_vp, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                       _vp, ctypes.c_int, ctypes.c_long, _vp, ctypes.c_int, ctypes.c_long, _vp,
                       ctypes.c_int, ctypes.c_long, ctypes.c_int],
    "dcn_roi_pool_fwd": [_vp, ctypes.POINTER(RoiDesc), _vp, _vp, _vp, _vp],
    "dcn_roi_pool_bwd": [_vp, ctypes.POINTER(RoiDesc), _vp, _vp, _vp, _vp, _vp, _vp],
    "dcn_roi_pool_fwd_host": [_vp, ctypes.POINTER(RoiDesc), _vp, _vp, _vp, _vp],
    "dcn_roi_pool_bwd_host": [_vp, ctypes.POINTER(RoiDesc), _vp, _vp, _vp, _vp, _vp, _vp],
}
_RESTYPES = {"dcn_last_error": ctypes.c_char_p}

_lib = None
_lock = threading.Lock()


def _one_hip_runtime():
    """torch-rocm bundles its own HIP runtime (torch/lib/libamdhip64.so, NEEDed unversioned),
    while libdcn NEEDs libamdhip64.so.7 (RUNPATH /opt/rocm/lib). Loaded first, libdcn maps
    /opt/rocm's runtime, and a torch imported later maps its own beside it: two HIP runtimes
    in one process (torch's streams handed to libdcn are then foreign objects; r02: heap
    corruption in a test that imported torch after libdcn). Loaded after torch, libdcn's
    NEEDED name matches torch's runtime (same soname) and the process keeps one. So where
    torch is installed it is imported before libdcn; torch-free callers (the Jittor / NumPy
    path) are unaffected. DCN_NO_TORCH_PRELOAD=1 skips this."""
    if "torch" in sys.modules or os.environ.get("DCN_NO_TORCH_PRELOAD") == "1":
        return
    try:
        import importlib.util
        if importlib.util.find_spec("torch") is None:
            return
    except (ImportError, ValueError):
        return
    import torch  # noqa: F401


def load(path: str | None = None):
    """Load libdcn.so and declare every prototype. Raises if it is missing."""
    _one_hip_runtime()
    global _lib
    with _lock:
        if _lib is not None and path is None:
            return _lib
        p = path or LIB_PATH
        if not os.path.exists(p):
            raise RuntimeError(f"libdcn.so not found at {p}: build it with "
                               f"`python -c 'import __graft_entry__ as g; g.build()'` "
                               f"(no CPU fallback exists)")
        L = ctypes.CDLL(p)
        for name, args in SIGNATURES.items():
            fn = getattr(L, name)
            fn.argtypes = args
            fn.restype = _RESTYPES.get(name, ctypes.c_int)
        if L.dcn_abi_version() != ABI_VERSION:
            raise RuntimeError("libdcn ABI version mismatch")
        if path is None:
            _lib = L
        return L


def last_error() -> str:
    msg = load().dcn_last_error()
    return msg.decode() if msg else ""


def check(rc: int, what: str = "libdcn"):
    if rc != 0:
        raise RuntimeError(f"{what} failed (status {rc}): {last_error()}")


def make_desc(B, C, H, W, O, kernel_size, stride, padding, dilation=(1, 1), deform_groups=1,
              bias=True, dtype=DCN_F32) -> Desc:
    return Desc(B, C, H, W, O, kernel_size[0], kernel_size[1], stride[0], stride[1], padding[0],
                padding[1], dilation[0], dilation[1], deform_groups, dtype, int(bool(bias)))


def make_roi_desc(feature_shape, num_rois, output_size, spatial_scale=1.0, ps=False,
                  part_size=None, trans_std=0.1, no_trans=False) -> RoiDesc:
    B, C, H, W = feature_shape
    ph, pw = output_size
    part_h, part_w = part_size if part_size else (0, 0)
    return RoiDesc(B, C, H, W, num_rois, ph, pw, part_h, part_w, float(spatial_scale),
                   float(trans_std), int(bool(ps)), int(bool(no_trans)))


def out_shape(desc: Desc):
    ho, wo = ctypes.c_int(), ctypes.c_int()
    check(load().dcn_out_shape(ctypes.byref(desc), ctypes.byref(ho), ctypes.byref(wo)),
          "dcn_out_shape")
    return ho.value, wo.value


def workspace_bytes(desc: Desc, with_backward) -> int:
    """dcn_workspace_bytes: with_backward False / True, or DCN_WS_FORWARD_NO_COLUMNS (2)."""
    n = ctypes.c_size_t()
    check(load().dcn_workspace_bytes(ctypes.byref(desc), int(with_backward), ctypes.byref(n)),
          "dcn_workspace_bytes")
    return n.value


def device_count() -> int:
    n = ctypes.c_int()
    rc = load().dcn_device_count(ctypes.byref(n))
    return n.value if rc == 0 else 0


class Handle:
    """One dcn_handle (device + stream + rocBLAS handle). Not thread-safe."""

    def __init__(self, device: int = 0):
        self.lib = load()
        h = ctypes.c_void_p()
        check(self.lib.dcn_create(int(device), ctypes.byref(h)), "dcn_create")
        self.h = h
        self.device = device
        # host-pointer API: bumped by every dcn_forward_host / dcn_backward_host call, so a
        # backward knows whether its forward's device state is still the handle's latest
        self.host_seq = 0

    def close(self):
        if getattr(self, "h", None):
            self.lib.dcn_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # --- streams / memory -----------------------------------------------------
    def set_stream(self, stream_ptr: int | None):
        """Bind to a hipStream_t handle; 0 / None is the HIP null stream (torch's default
        stream reports 0). use_own_stream() returns to the handle's own stream."""
        check(self.lib.dcn_set_stream(self.h, ctypes.c_void_p(stream_ptr or 0)), "dcn_set_stream")

    def use_own_stream(self):
        check(self.lib.dcn_use_own_stream(self.h), "dcn_use_own_stream")

    def synchronize(self):
        check(self.lib.dcn_synchronize(self.h), "dcn_synchronize")

    def malloc(self, nbytes: int) -> int:
        p = ctypes.c_void_p()
        check(self.lib.dcn_malloc(self.h, nbytes, ctypes.byref(p)), "dcn_malloc")
        return p.value

    def free(self, ptr: int):
        check(self.lib.dcn_free(self.h, ctypes.c_void_p(ptr)), "dcn_free")

    def h2d(self, dst: int, arr):
        check(self.lib.dcn_memcpy_h2d(self.h, ctypes.c_void_p(dst), arr.ctypes.data_as(_vp),
                                      arr.nbytes), "dcn_memcpy_h2d")

    def d2h(self, arr, src: int):
        check(self.lib.dcn_memcpy_d2h(self.h, arr.ctypes.data_as(_vp), ctypes.c_void_p(src),
                                      arr.nbytes), "dcn_memcpy_d2h")

    # --- GEMM arithmetic (include/dcn.h dcn_math) ---------------------------------
    def set_math(self, math: int):
        """0 native f32 MFMA; 3 / 6 / 9 split-bf16 products (DCN_MATH_F32_BF16X*)."""
        check(self.lib.dcn_set_math(self.h, int(math)), "dcn_set_math")

    def set_fwd_path(self, path: int):
        """0 DCN_FWD_AUTO (measured-faster schedule), 1 DCN_FWD_UNFUSED, 2 DCN_FWD_FUSED,
        3 DCN_FWD_FUSED_NOCOL (DCN_BF16: no columns written)."""
        check(self.lib.dcn_set_fwd_path(self.h, int(path)), "dcn_set_fwd_path")

    def get_fwd_path(self) -> int:
        p = ctypes.c_int()
        check(self.lib.dcn_get_fwd_path(self.h, ctypes.byref(p)), "dcn_get_fwd_path")
        return p.value

    # --- data-parallel gradient exchange (include/dcn.h) ---------------------------
    def set_comm(self, comm):
        """Attach a dcn_dp.RcclComm (None detaches): dcn_backward then returns gradients
        summed over the ranks, the ∂W/∂b all-reduce overlapped with the rest of it."""
        check(self.lib.dcn_set_comm(self.h, comm.c if comm is not None else None), "dcn_set_comm")

    def set_grad_stream(self, stream_ptr: int | None):
        """Each later dcn_backward makes this hipStream_t wait until ∂W and ∂b are final
        (None / 0 disables), so a collective enqueued on it overlaps the backward's rest."""
        check(self.lib.dcn_set_grad_stream(self.h, ctypes.c_void_p(stream_ptr or 0)),
              "dcn_set_grad_stream")

    def get_math(self) -> int:
        m = ctypes.c_int()
        check(self.lib.dcn_get_math(self.h, ctypes.byref(m)), "dcn_get_math")
        return m.value

    # --- profiling -------------------------------------------------------------
    def prof_enable(self, capacity: int):
        check(self.lib.dcn_prof_enable(self.h, int(capacity)), "dcn_prof_enable")

    def prof_read(self, kernel: str):
        t, n = ctypes.c_double(), ctypes.c_int()
        check(self.lib.dcn_prof_read(self.h, KERNEL_IDS[kernel], ctypes.byref(t), ctypes.byref(n)),
              "dcn_prof_read")
        return t.value, n.value

    def prof_reset(self):
        check(self.lib.dcn_prof_reset(self.h), "dcn_prof_reset")


class HostState:
    """One dcn_host_state (include/dcn.h): a module's device copies of x / offsets / weights
    and its own workspace on `handle`, so its backward reuses its forward's columns whatever
    other modules ran on the handle in between. Keeps the handle alive."""

    def __init__(self, handle: Handle, chunks: int = 0):
        self.handle, self.lib = handle, handle.lib
        s = ctypes.c_void_p()
        check(self.lib.dcn_host_state_create(handle.h, ctypes.byref(s)), "dcn_host_state_create")
        self.s = s
        self.host_seq = 0  # bumped by every call on this state (see HostFwdCtx)
        if chunks:
            self.set_chunks(chunks)

    def set_chunks(self, chunks: int):
        """Image chunks of the transfer pipeline: 0 = auto, else min(chunks, B, 16)."""
        check(self.lib.dcn_host_state_set_chunks(self.s, int(chunks)), "dcn_host_state_set_chunks")

    def close(self):
        if getattr(self, "s", None):
            self.lib.dcn_host_state_destroy(self.s)
            self.s = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def ptr(a):
    """Host pointer of a C-contiguous float32 numpy array (None -> NULL)."""
    if a is None:
        return None
    if a.dtype.name != "float32" or not a.flags.c_contiguous:
        raise TypeError("libdcn expects C-contiguous float32 arrays")
    return a.ctypes.data_as(_vp)


_default = {}


def default_handle(device: int | None = None) -> Handle:
    """Process-wide handle per device (DCN_DEVICE env var selects the default)."""
    dev = int(os.environ.get("DCN_DEVICE", "0")) if device is None else int(device)
    key = (threading.get_ident(), dev)
    h = _default.get(key)
    if h is None:
        h = _default[key] = Handle(dev)
    return h
