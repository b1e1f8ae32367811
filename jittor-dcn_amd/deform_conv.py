"""Drop-in replacement for the reference's `deform_conv.DeformConv2d`.

Callers keep their import line unchanged (train.py:299, test.py:12):

    import sys; sys.path.insert(0, "<repo>/jittor-dcn_amd")
    from deform_conv import DeformConv2d
    conv = DeformConv2d(16, 32, 3, 2, 1)          # train.py:311

Surface kept from /root/reference/deform_conv.py:6-81:
  * constructor (in_channels, out_channels, kernel_size=3, stride=1, padding=1,
    bias=True) (:7); kernel_size/stride/padding normalised to tuples (:11-13);
  * attributes in_channels, out_channels, kernel_size, stride, padding, N (:9-14);
  * parameters offset_conv.weight [2N, C, kh, kw], offset_conv.bias [2N] (zero
    init, :16-21, :27-28), weight [O, C, kh, kw] ~ N(0, sqrt(2/(C*kh*kw))) (:23-24),
    bias [O] zero or None (:25) — so state-dict keys round-trip (train.py:461,
    test.py:19);
  * execute(x) -> [B, O, H_out, W_out] (:56-81), reached through __call__.

Compute: every call goes to libdcn.so (hand-written gfx950 HIP kernels + rocBLAS)
through ctypes (dcn_runtime.py). There is no CPU fallback: without the library
or a HIP device, execute() raises RuntimeError.

Backends:
  * Jittor importable  -> a jt.nn.Module whose execute() is a jt.Function, so the
    gradients reach Jittor autodiff / optimizer.backward (train.py:414).
  * otherwise          -> a NumPy module: execute(x) returns a NumPy array and
    backward(grad_out) fills `.grad` on the four parameters and returns ∂x.
"""
from __future__ import annotations

import ctypes
import math

import numpy as np

import dcn_runtime as rt
import hostmem

try:  # pragma: no cover - Jittor is not installable in the build image
    import jittor as jt
    from jittor import nn as jnn
    HAVE_JITTOR = True
except Exception:  # ImportError or a broken jittor install
    jt = None
    HAVE_JITTOR = False


def _pair(v):
    return v if isinstance(v, tuple) else (v, v)


def _f32(a):
    return np.ascontiguousarray(a, dtype=np.float32)


class HostFwdCtx:
    """What a dcn_backward_numpy needs to reuse its forward's device state (libdcn's
    DCN_HOST_REUSE_FWD): the host state (a module's rt.HostState, or the handle's own) the
    forward ran on, the exact arrays it uploaded and the state's call sequence number at the
    time. Reuse happens only when no other call ran on that state since."""

    __slots__ = ("owner", "seq", "arrays")

    def __init__(self, owner, seq, x, w_off, w, off):
        # the arrays themselves stay referenced (their memory cannot be recycled meanwhile);
        # they are matched by data pointer, as the library checks them
        self.owner, self.seq, self.arrays = owner, seq, (x, w_off, w, off)

    def matches(self, owner, x, w_off, w, off):
        return (self.owner is owner and self.seq == owner.host_seq
                and all(a.ctypes.data == b.ctypes.data and a.shape == b.shape
                        for a, b in zip(self.arrays, (x, w_off, w, off))))


def dcn_forward_numpy(x, w_off, b_off, w, b, stride, padding, handle=None, return_ctx=False,
                      state=None):
    """out, off = DeformConv2d.execute on host arrays (one libdcn call). state: a
    rt.HostState (one per module; or a callable returning it) to run on instead of the
    handle's own. With return_ctx,
    also a HostFwdCtx for dcn_backward_numpy(ctx=...)."""
    x, w_off, b_off, w = _f32(x), _f32(w_off), _f32(b_off), _f32(w)
    b = None if b is None else _f32(b)
    B, C, H, W = x.shape
    O, Cw, kh, kw = w.shape
    if Cw != C:
        raise ValueError(f"input has {C} channels, weight expects {Cw}")
    if B == 0:  # empty batch: empty outputs, as the reference's ops give (no launch)
        Ho, Wo = rt.out_shape(rt.make_desc(1, C, H, W, O, (kh, kw), stride, padding))
        out = np.empty((0, O, Ho, Wo), np.float32)
        off = np.empty((0, w_off.shape[0], Ho, Wo), np.float32)
        # no forward state to reuse: dcn_backward_numpy takes ctx=None (and B == 0 there too)
        return (out, off, None) if return_ctx else (out, off)
    # after the empty-batch case: it launches nothing
    if callable(state):  # a module's host_state, resolved only when there is work
        state = state()
    h = state.handle if state is not None else (handle or rt.default_handle())
    desc = rt.make_desc(B, C, H, W, O, (kh, kw), stride, padding, bias=b is not None)
    Ho, Wo = rt.out_shape(desc)
    hostmem.use_pinned(h)  # page-locked result blocks: their downloads are DMAs
    out = hostmem.empty((B, O, Ho, Wo))
    off = hostmem.empty((B, w_off.shape[0], Ho, Wo))
    owner = state if state is not None else h
    owner.host_seq += 1
    args = (desc, rt.ptr(x), rt.ptr(w_off), rt.ptr(b_off), rt.ptr(w), rt.ptr(b), rt.ptr(out),
            rt.ptr(off))
    if state is not None:
        rt.check(h.lib.dcn_forward_host_s(state.s, *args), "dcn_forward_host_s")
    else:
        rt.check(h.lib.dcn_forward_host(h.h, *args), "dcn_forward_host")
    if return_ctx:
        return out, off, HostFwdCtx(owner, owner.host_seq, x, w_off, w, off)
    return out, off


def dcn_backward_numpy(x, off, w_off, w, has_bias, grad_out, stride, padding, handle=None,
                       ctx=None, state=None, offset_grad=True):
    """Grads of DeformConv2d.execute (dict keyed like the state dict, plus 'x' and, with
    offset_grad, 'offset'). ctx: the forward's HostFwdCtx; when nothing else ran on its
    host state since, x / off / weights are not uploaded again and the forward's columns
    are reused. state: the rt.HostState to run on (default: ctx's, else the handle's)."""
    x, off, w_off, w, grad_out = map(_f32, (x, off, w_off, w, grad_out))
    B, C, H, W = x.shape
    O, _, kh, kw = w.shape
    if B == 0:  # empty batch: nothing sampled, every parameter gradient is zero
        g = {"x": np.empty_like(x), "weight": np.zeros_like(w),
             "offset_conv.weight": np.zeros_like(w_off),
             "offset_conv.bias": np.zeros(w_off.shape[0], np.float32)}
        if offset_grad:
            g["offset"] = np.empty_like(off)
        if has_bias:
            g["bias"] = np.zeros(O, np.float32)
        return g
    if callable(state):
        state = state()
    if state is None and ctx is not None and isinstance(ctx.owner, rt.HostState):
        state = ctx.owner
    h = state.handle if state is not None else (
        handle or (ctx.owner if ctx is not None else rt.default_handle()))
    owner = state if state is not None else h
    desc = rt.make_desc(B, C, H, W, O, (kh, kw), stride, padding, bias=has_bias)
    hostmem.use_pinned(h)
    g = {"x": hostmem.empty_like(x), "weight": hostmem.empty_like(w),
         "offset_conv.weight": hostmem.empty_like(w_off),
         "offset_conv.bias": np.empty(w_off.shape[0], np.float32)}
    if offset_grad:
        g["offset"] = hostmem.empty_like(off)
    gb = np.empty(O, np.float32) if has_bias else None
    flags = rt.HOST_REUSE_FWD if ctx is not None and ctx.matches(owner, x, w_off, w, off) else 0
    owner.host_seq += 1
    args = (desc, rt.ptr(x), rt.ptr(off), rt.ptr(w_off), rt.ptr(w), rt.ptr(grad_out),
            rt.ptr(g["x"]), rt.ptr(g["weight"]), rt.ptr(gb), rt.ptr(g["offset_conv.weight"]),
            rt.ptr(g["offset_conv.bias"]), rt.ptr(g.get("offset")), flags)
    if state is not None:
        rt.check(h.lib.dcn_backward_host_s(state.s, *args), "dcn_backward_host_s")
    else:
        rt.check(h.lib.dcn_backward_host_ex(h.h, *args), "dcn_backward_host_ex")
    if has_bias:
        g["bias"] = gb
    return g


def _roi_args(features, rois, offsets, output_size, ps, no_trans):
    features, rois = _f32(features), _f32(rois)
    R = rois.shape[0]
    P = output_size[0] * output_size[1]
    if rois.ndim != 2 or rois.shape[1] != 5:
        raise ValueError(f"rois must be [R, 5], got {rois.shape}")
    if ps and no_trans:
        offsets = None
    elif ps:  # offsets[:, part_idx*2 (+1)] (deform_conv.py:198-199): the first 2P columns
        offsets = _f32(np.asarray(offsets, np.float32).reshape(R, -1)[:, :2 * P])
    else:  # offsets[:, p, 0/1] (deform_conv.py:113-114)
        offsets = _f32(np.asarray(offsets, np.float32).reshape(R, -1, 2)[:, :P])
    return features, rois, offsets


def roi_pool_forward_numpy(features, rois, offsets, output_size, spatial_scale=1.0, ps=False,
                           part_size=None, trans_std=0.1, no_trans=False, handle=None):
    """The reference's value before its final reshape: the bilinear corner sums over all
    bins, [R, C] (DeformRoIPool, deform_conv.py:92-157) or [R, C // (ph*pw)]
    (DeformPSRoIPool, :174-239). One libdcn call."""
    h = handle or rt.default_handle()
    features, rois, offsets = _roi_args(features, rois, offsets, output_size, ps, no_trans)
    d = rt.make_roi_desc(features.shape, rois.shape[0], output_size, spatial_scale, ps, part_size,
                         trans_std, no_trans)
    P = output_size[0] * output_size[1]
    Cout = features.shape[1] // P if ps else features.shape[1]
    out = np.empty((rois.shape[0], Cout), np.float32)
    rt.check(h.lib.dcn_roi_pool_fwd_host(h.h, ctypes.byref(d), rt.ptr(features), rt.ptr(rois),
                                         rt.ptr(offsets), rt.ptr(out)), "dcn_roi_pool_fwd_host")
    return out


def roi_pool_backward_numpy(features, rois, offsets, grad_out, output_size, spatial_scale=1.0,
                            ps=False, part_size=None, trans_std=0.1, no_trans=False,
                            handle=None):
    """(∂features, ∂offsets) of roi_pool_forward_numpy; ∂offsets has the caller's offsets
    shape (zeros when the PS pool ignores them). The RoI boxes get no gradient."""
    h = handle or rt.default_handle()
    offsets_in = offsets
    features, rois, offsets = _roi_args(features, rois, offsets, output_size, ps, no_trans)
    d = rt.make_roi_desc(features.shape, rois.shape[0], output_size, spatial_scale, ps, part_size,
                         trans_std, no_trans)
    R, P = rois.shape[0], output_size[0] * output_size[1]
    gf = np.empty_like(features)
    goff = np.zeros((R, P, 2), np.float32)
    rt.check(h.lib.dcn_roi_pool_bwd_host(h.h, ctypes.byref(d), rt.ptr(features), rt.ptr(rois),
                                         rt.ptr(offsets), rt.ptr(_f32(grad_out)), rt.ptr(gf),
                                         rt.ptr(goff)), "dcn_roi_pool_bwd_host")
    g_in = np.zeros(np.shape(offsets_in), np.float32) if offsets_in is not None else None
    if g_in is not None:
        flat = g_in.reshape(R, -1)
        flat[:, :2 * P] = goff.reshape(R, 2 * P)
    return gf, g_in


# ---------------------------------------------------------------------------
# NumPy backend
# ---------------------------------------------------------------------------
class Parameter(np.ndarray):
    """float32 ndarray with a `.grad` slot (what Adam in train.py:350 iterates)."""

    def __new__(cls, data):
        obj = np.ascontiguousarray(data, dtype=np.float32).view(cls)
        obj.grad = None
        return obj

    def __array_finalize__(self, obj):
        self.grad = getattr(obj, "grad", None)


class Module:
    """Minimal module protocol: parameters / state_dict / load_state_dict / __call__."""

    def __init__(self):
        self.training = True

    def _children(self):
        return [(k, v) for k, v in vars(self).items() if isinstance(v, Module)]

    def named_parameters(self, prefix=""):
        for k, v in vars(self).items():
            if isinstance(v, Parameter):
                yield prefix + k, v
        for k, m in self._children():
            yield from m.named_parameters(prefix + k + ".")

    def parameters(self):
        return [p for _, p in self.named_parameters()]

    def state_dict(self):
        return {k: np.array(v) for k, v in self.named_parameters()}

    def load_state_dict(self, sd):
        for k, v in sd.items():
            obj, *path = [self] + k.split(".")
            for part in path[:-1]:
                obj = getattr(obj, part)
            cur = getattr(obj, path[-1])
            v = np.asarray(v, np.float32)
            if cur is not None and tuple(cur.shape) != tuple(v.shape):
                raise ValueError(f"shape mismatch for {k}: {cur.shape} vs {v.shape}")
            setattr(obj, path[-1], Parameter(v))

    def load(self, path):
        """Like jt.Module.load (test.py:19) for .npz state dicts."""
        with np.load(path, allow_pickle=False) as z:
            self.load_state_dict({k: z[k] for k in z.files})

    def save(self, path):
        np.savez(path, **self.state_dict())

    def zero_grad(self):
        for p in self.parameters():
            p.grad = None

    def train(self):
        self.training = True

    def eval(self):
        self.training = False

    def __call__(self, *a, **k):
        return self.execute(*a, **k)


class Conv(Module):
    """Parameter holder for `offset_conv` (nn.Conv in deform_conv.py:16-21). Its
    math runs fused inside libdcn (dcn_forward); it is never executed alone."""

    def __init__(self, in_channels, out_channels, kernel_size, stride, padding):
        super().__init__()
        self.in_channels, self.out_channels = in_channels, out_channels
        self.kernel_size, self.stride, self.padding = kernel_size, stride, padding
        self.weight = Parameter(np.zeros((out_channels, in_channels, *kernel_size), np.float32))
        self.bias = Parameter(np.zeros(out_channels, np.float32))


class DeformConv2dNumpy(Module):
    """DeformConv2d (deform_conv.py:6-81) over NumPy arrays, computed by libdcn."""

    def __init__(self, in_channels, out_channels, kernel_size=3, stride=1, padding=1, bias=True,
                 seed=None):
        super().__init__()
        self.in_channels = in_channels
        self.out_channels = out_channels
        self.kernel_size = _pair(kernel_size)
        self.stride = _pair(stride)
        self.padding = _pair(padding)
        self.N = self.kernel_size[0] * self.kernel_size[1]
        self.offset_conv = Conv(in_channels, 2 * self.N, self.kernel_size, self.stride, self.padding)
        std = math.sqrt(2.0 / (in_channels * self.kernel_size[0] * self.kernel_size[1]))
        rng = np.random.default_rng(seed)
        self.weight = Parameter(rng.normal(0.0, std, (out_channels, in_channels, *self.kernel_size)))
        self.bias = Parameter(np.zeros(out_channels, np.float32)) if bias else None
        self._ctx = None
        self._hstate = None

    def host_state(self):
        """This module's device state (rt.HostState on the thread's default handle): its
        backward reuses its own forward's columns however many modules share the handle."""
        h = rt.default_handle()
        if self._hstate is None or self._hstate.handle is not h:
            self._hstate = rt.HostState(h)
        return self._hstate

    def execute(self, x):
        x = _f32(x)
        out, off, hctx = dcn_forward_numpy(x, self.offset_conv.weight, self.offset_conv.bias,
                                           self.weight, self.bias, self.stride, self.padding,
                                           return_ctx=True, state=self.host_state)
        self._ctx = (x, off, hctx) if self.training else None
        return out

    def backward(self, grad_out):
        """Accumulate parameter grads (.grad) and return ∂L/∂x."""
        if self._ctx is None:
            raise RuntimeError("backward() needs a preceding execute() in training mode")
        x, off, hctx = self._ctx
        g = dcn_backward_numpy(x, off, self.offset_conv.weight, self.weight, self.bias is not None,
                               grad_out, self.stride, self.padding, ctx=hctx,
                               state=self.host_state, offset_grad=False)
        for name, p in self.named_parameters():
            p.grad = g[name] if p.grad is None else p.grad + g[name]
        return g["x"]


class _RoIPoolBase(Module):
    """Shared execute/backward of the two RoI pools (NumPy backend). Like the reference
    (deform_conv.py:158, :241), execute() reshapes the bin sum to [R, C, ph, pw], which
    raises for ph*pw != 1 exactly where the reference's reshape does."""

    _ps = False

    def _kw(self):
        return {}

    def execute(self, features, rois, offsets):
        s = roi_pool_forward_numpy(features, rois, offsets, self.output_size, self.spatial_scale,
                                   ps=self._ps, **self._kw())
        out = s.reshape(np.shape(rois)[0], s.shape[1], *self.output_size)  # :158 / :241
        if self.training:
            self._ctx = (features, rois, offsets)
        return out

    def backward(self, grad_out):
        """(∂features, ∂offsets) for ∂out of execute's shape."""
        if getattr(self, "_ctx", None) is None:
            raise RuntimeError("backward() needs a preceding execute() in training mode")
        features, rois, offsets = self._ctx
        g = np.asarray(grad_out, np.float32).reshape(np.shape(rois)[0], -1)
        return roi_pool_backward_numpy(features, rois, offsets, g, self.output_size,
                                       self.spatial_scale, ps=self._ps, **self._kw())


class DeformRoIPoolNumpy(_RoIPoolBase):
    """deform_conv.py:85-159: DeformRoIPool(output_size, spatial_scale=1.0,
    sampling_ratio=1) on libdcn (sampling_ratio is stored, unused, as in the reference)."""

    def __init__(self, output_size, spatial_scale=1.0, sampling_ratio=1):
        super().__init__()
        self.output_size = output_size if isinstance(output_size, tuple) else (output_size,
                                                                              output_size)
        self.spatial_scale = spatial_scale
        self.sampling_ratio = sampling_ratio


class DeformPSRoIPoolNumpy(_RoIPoolBase):
    """deform_conv.py:162-241: DeformPSRoIPool(output_size, spatial_scale=1.0,
    sampling_ratio=1, no_trans=False, group_size=1, part_size=None, trans_std=0.1)."""

    _ps = True

    def __init__(self, output_size, spatial_scale=1.0, sampling_ratio=1, no_trans=False,
                 group_size=1, part_size=None, trans_std=0.1):
        super().__init__()
        self.output_size = output_size if isinstance(output_size, tuple) else (output_size,
                                                                              output_size)
        self.spatial_scale = spatial_scale
        self.sampling_ratio = sampling_ratio
        self.no_trans = no_trans
        self.group_size = group_size
        self.part_size = part_size if part_size else self.output_size
        self.trans_std = trans_std

    def _kw(self):
        return dict(part_size=self.part_size, trans_std=self.trans_std, no_trans=self.no_trans)


# ---------------------------------------------------------------------------
# Jittor backend (exercised only where jittor imports; not in the build image)
# ---------------------------------------------------------------------------
if HAVE_JITTOR:  # pragma: no cover

    class _DCNFunction(jt.Function):
        """jt.Function whose execute/grad call libdcn; inputs are the module's Vars so
        Jittor autodiff routes gradients to offset_conv.{weight,bias}, weight, bias."""

        def execute(self, x, w_off, b_off, w, b, stride, padding, state):
            self.stride, self.padding, self.state = stride, padding, state
            self.has_bias = b is not None
            xn, won, wn = x.numpy(), w_off.numpy(), w.numpy()
            xn, won, wn = _f32(xn), _f32(won), _f32(wn)
            out, off, hctx = dcn_forward_numpy(xn, won, b_off.numpy(), wn,
                                               None if b is None else b.numpy(), stride, padding,
                                               return_ctx=True, state=state)
            self.saved = (xn, off, won, wn, hctx)
            return jt.array(out)

        def grad(self, grad_out):
            xn, off, won, wn, hctx = self.saved
            g = dcn_backward_numpy(xn, off, won, wn, self.has_bias, grad_out.numpy(),
                                   self.stride, self.padding, ctx=hctx, state=self.state,
                                   offset_grad=False)
            gb = jt.array(g["bias"]) if self.has_bias else None
            return (jt.array(g["x"]), jt.array(g["offset_conv.weight"]),
                    jt.array(g["offset_conv.bias"]), jt.array(g["weight"]), gb, None, None,
                    None)

    class DeformConv2d(jnn.Module):
        def __init__(self, in_channels, out_channels, kernel_size=3, stride=1, padding=1,
                     bias=True):
            super().__init__()
            self.in_channels = in_channels
            self.out_channels = out_channels
            self.kernel_size = _pair(kernel_size)
            self.stride = _pair(stride)
            self.padding = _pair(padding)
            self.N = self.kernel_size[0] * self.kernel_size[1]
            self.offset_conv = jnn.Conv(in_channels, 2 * self.N, kernel_size=self.kernel_size,
                                        stride=self.stride, padding=self.padding)
            std = math.sqrt(2.0 / (in_channels * self.kernel_size[0] * self.kernel_size[1]))
            self.weight = jt.init.gauss([out_channels, in_channels, *self.kernel_size], mean=0.0,
                                        std=std)
            self.bias = jt.init.constant(shape=[out_channels], value=0.0) if bias else None
            self.offset_conv.weight = jt.zeros_like(self.offset_conv.weight)
            self.offset_conv.bias = jt.zeros_like(self.offset_conv.bias)
            self._hstate = None

        host_state = DeformConv2dNumpy.host_state

        def execute(self, x):
            return _DCNFunction.apply(x, self.offset_conv.weight, self.offset_conv.bias,
                                      self.weight, self.bias, self.stride, self.padding,
                                      self.host_state)
    class _RoIPoolFunction(jt.Function):
        """jt.Function for both RoI pools: ∂features and ∂offsets reach Jittor autodiff
        (the boxes get none, as they come from the data)."""

        def execute(self, features, rois, offsets, module):
            self.m = module
            self.saved = (features.numpy(), rois.numpy(),
                          None if offsets is None else offsets.numpy())
            s = roi_pool_forward_numpy(*self.saved, module.output_size, module.spatial_scale,
                                       ps=module._ps, **module._kw())
            return jt.array(s.reshape(rois.shape[0], s.shape[1], *module.output_size))

        def grad(self, grad_out):
            f, r, o = self.saved
            m = self.m
            gf, go = roi_pool_backward_numpy(f, r, o, grad_out.numpy().reshape(r.shape[0], -1),
                                             m.output_size, m.spatial_scale, ps=m._ps, **m._kw())
            return jt.array(gf), None, None if go is None else jt.array(go), None

    class DeformRoIPool(jnn.Module):
        _ps = False
        _kw = DeformRoIPoolNumpy._kw

        def __init__(self, output_size, spatial_scale=1.0, sampling_ratio=1):
            super().__init__()
            self.output_size = output_size if isinstance(output_size, tuple) else (
                output_size, output_size)
            self.spatial_scale = spatial_scale
            self.sampling_ratio = sampling_ratio

        def execute(self, features, rois, offsets):
            return _RoIPoolFunction.apply(features, rois, offsets, self)

    class DeformPSRoIPool(jnn.Module):
        _ps = True
        _kw = DeformPSRoIPoolNumpy._kw

        def __init__(self, output_size, spatial_scale=1.0, sampling_ratio=1, no_trans=False,
                     group_size=1, part_size=None, trans_std=0.1):
            super().__init__()
            self.output_size = output_size if isinstance(output_size, tuple) else (
                output_size, output_size)
            self.spatial_scale = spatial_scale
            self.sampling_ratio = sampling_ratio
            self.no_trans = no_trans
            self.group_size = group_size
            self.part_size = part_size if part_size else self.output_size
            self.trans_std = trans_std

        def execute(self, features, rois, offsets):
            return _RoIPoolFunction.apply(features, rois, offsets, self)
else:
    DeformConv2d = DeformConv2dNumpy
    DeformRoIPool = DeformRoIPoolNumpy
    DeformPSRoIPool = DeformPSRoIPoolNumpy

__all__ = ["DeformConv2d", "DeformConv2dNumpy", "DeformRoIPool", "DeformRoIPoolNumpy",
           "DeformPSRoIPool", "DeformPSRoIPoolNumpy", "dcn_forward_numpy", "dcn_backward_numpy",
           "HostFwdCtx",
           "roi_pool_forward_numpy", "roi_pool_backward_numpy", "HAVE_JITTOR"]
