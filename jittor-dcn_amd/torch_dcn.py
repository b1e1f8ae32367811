"""DeformConv2d for PyTorch callers: libdcn's device API as a torch.autograd.Function.

The reference's operator surface (deform_conv.py:6-28: DeformConv2d(in_channels,
out_channels, kernel_size=3, stride=1, padding=1, bias=True), zero-initialised offset
conv, gauss-initialised weight) over GPU-resident torch tensors. Forward and backward
are dcn_forward / dcn_backward on torch's current HIP stream, so there are no host
copies. Each module keeps its workspace, so the backward reuses the forward's columns
(DCN_BWD_COL_IN_WS); a bf16 forward that no backward will follow (torch.no_grad, or no
input needing a gradient: the reference's jt.no_grad inference, train.py:430) calls
dcn_forward_ex with DCN_FWD_NO_COLUMNS, which writes no column matrix and leaves the shared
handle's forward path alone. torch is only the tensor container
here: every kernel is libdcn's, and a missing libdcn.so or HIP device raises (no fallback).
"""
from __future__ import annotations

import math

import torch

import dcn_runtime as rt

_handles = {}


def _handle(dev: torch.device) -> rt.Handle:
    idx = dev.index if dev.index is not None else torch.cuda.current_device()
    h = _handles.get(idx)
    if h is None:
        h = _handles[idx] = rt.Handle(idx)
    h.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    return h


def _pair(v):
    return tuple(v) if isinstance(v, (tuple, list)) else (v, v)


_DT = {torch.float32: rt.DCN_F32, torch.bfloat16: rt.DCN_BF16}


class _Workspace:
    """Per-module device workspace (grown on demand, kept across steps). `fwd_count`
    tells a backward whether the columns in it are still its own forward's."""

    def __init__(self):
        self.buf = None
        self.fwd_count = 0

    def get(self, nbytes: int, dev: torch.device) -> torch.Tensor:
        if self.buf is None or self.buf.numel() < nbytes or self.buf.device != dev:
            self.buf = torch.empty(nbytes, dtype=torch.uint8, device=dev)
        return self.buf


class DeformConv2dFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w_off, b_off, w, b, stride, padding, ws: _Workspace, nocol=False):
        if x.dtype not in _DT:
            raise TypeError("libdcn DeformConv2d takes float32 or bfloat16 tensors")
        x, w_off, b_off, w = (t.contiguous() for t in (x, w_off, b_off, w))
        b = b.contiguous() if b is not None else None
        B, C, H, W = x.shape
        O, _, kh, kw = w.shape
        desc = rt.make_desc(B, C, H, W, O, (kh, kw), stride, padding, bias=b is not None,
                            dtype=_DT[x.dtype])
        Ho, Wo = rt.out_shape(desc)
        h = _handle(x.device)
        out = torch.empty(B, O, Ho, Wo, device=x.device, dtype=x.dtype)
        off = torch.empty(B, w_off.shape[0], Ho, Wo, device=x.device, dtype=x.dtype)
        wsb = rt.workspace_bytes(desc, True)
        buf = ws.get(wsb, x.device)
        P = lambda t: None if t is None else t.data_ptr()
        # forward-only (no backward will read the columns): a per-call flag,
        # so the handle shared by every module on this device keeps the caller's path
        flags = rt.DCN_FWD_NO_COLUMNS if nocol else 0
        rt.check(h.lib.dcn_forward_ex(h.h, desc, P(x), P(w_off), P(b_off), P(w), P(b), P(out),
                                      P(off), P(buf), wsb, flags), "dcn_forward_ex")
        ctx.save_for_backward(x, off, w_off, w)
        ctx.desc, ctx.ws, ctx.wsb, ctx.has_bias = desc, ws, wsb, b is not None
        ws.fwd_count += 1
        ctx.token = (ws.fwd_count, buf.data_ptr())
        return out

    @staticmethod
    def backward(ctx, gout):
        x, off, w_off, w = ctx.saved_tensors
        gout = gout.contiguous()
        h = _handle(x.device)
        gx, gw, gwo = torch.empty_like(x), torch.empty_like(w), torch.empty_like(w_off)
        gbo = torch.empty(w_off.shape[0], device=x.device, dtype=x.dtype)
        gb = torch.empty(w.shape[0], device=x.device, dtype=x.dtype) if ctx.has_bias else None
        buf = ctx.ws.get(ctx.wsb, x.device)
        # the columns are still in the workspace iff no other forward used it since
        flags = rt.DCN_BWD_COL_IN_WS if ctx.token == (ctx.ws.fwd_count, buf.data_ptr()) else 0
        P = lambda t: None if t is None else t.data_ptr()
        rt.check(h.lib.dcn_backward(h.h, ctx.desc, P(x), P(off), P(w_off), P(w), P(gout), P(gx),
                                    P(gw), P(gb), P(gwo), P(gbo), None, P(buf), ctx.wsb, flags),
                 "dcn_backward")
        return gx, gwo, gbo, gw, gb, None, None, None, None


class DeformConv2d(torch.nn.Module):
    """torch twin of deform_conv.py:6-81's module surface, computed by libdcn."""

    def __init__(self, in_channels, out_channels, kernel_size=3, stride=1, padding=1, bias=True):
        super().__init__()
        self.in_channels, self.out_channels = in_channels, out_channels
        self.kernel_size, self.stride, self.padding = (_pair(kernel_size), _pair(stride),
                                                       _pair(padding))
        kh, kw = self.kernel_size
        self.N = kh * kw
        self.offset_conv = torch.nn.Conv2d(in_channels, 2 * self.N, self.kernel_size,
                                           self.stride, self.padding)
        with torch.no_grad():  # deform_conv.py:27-28
            self.offset_conv.weight.zero_()
            self.offset_conv.bias.zero_()
        std = math.sqrt(2.0 / (in_channels * kh * kw))  # deform_conv.py:23-24
        self.weight = torch.nn.Parameter(torch.randn(out_channels, in_channels, kh, kw) * std)
        self.bias = torch.nn.Parameter(torch.zeros(out_channels)) if bias else None
        self._ws = _Workspace()

    def forward(self, x):
        params = (x, self.offset_conv.weight, self.offset_conv.bias, self.weight, self.bias)
        needs_grad = torch.is_grad_enabled() and any(
            t is not None and t.requires_grad for t in params)
        return DeformConv2dFunction.apply(x, self.offset_conv.weight, self.offset_conv.bias,
                                          self.weight, self.bias, self.stride, self.padding,
                                          self._ws, not needs_grad)
