"""Batch-sharded data parallelism for DeformConv2d.

Every image is independent in the forward pass and in ∂x / ∂offset, so B images are split
into contiguous per-rank shards with replicated parameters. The only exchange is ONE
in-place sum all-reduce per step of the four parameter gradients, packed into a single
flat fp32 buffer (∂W, ∂b, ∂W_off, ∂b_off = 631,570 values = 2.53 MB at config 3):
ring cost on 8 GPUs ≈ 2·(7/8)·2.53 MB per GPU over xGMI, tens of µs against a ~9 ms step.

The sum is what a loss summed over the global batch needs; a caller whose loss is a
mean over the global batch scales grad_out by 1/B_global before dcn_backward, exactly as
a single-device run would (the reference's train.py:414 optimizer.backward).

Two transports, same packing:
  * torch.distributed (backend "nccl" = RCCL on ROCm, or "gloo" on CPU) — bench.py;
  * libdcn's own RCCL communicator (dcn_comm_* / dcn_allreduce_grads in include/dcn.h)
    for a torch-free Jittor / NumPy caller.
"""
from __future__ import annotations

import ctypes

# Packing order of the flat gradient buffer (state-dict names, deform_conv.py:16-28).
PARAM_ORDER = ("weight", "bias", "offset_conv.weight", "offset_conv.bias")


def shard_range(batch: int, world: int, rank: int) -> tuple[int, int]:
    """Contiguous shard (first image, image count) of `batch` images for `rank`; the
    first batch % world ranks take one extra image."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f"rank {rank} outside world of {world}")
    q, r = divmod(batch, world)
    nb = q + (1 if rank < r else 0)
    b0 = rank * q + min(rank, r)
    return b0, nb


def param_shapes(C: int, O: int, kh: int, kw: int, bias: bool = True, deform_groups: int = 1):
    """Parameter shapes of DeformConv2d(C, O, (kh, kw)) in PARAM_ORDER (bias omitted
    when bias=False)."""
    J = 2 * kh * kw * deform_groups
    shapes = {"weight": (O, C, kh, kw), "bias": (O,), "offset_conv.weight": (J, C, kh, kw),
              "offset_conv.bias": (J,)}
    if not bias:
        del shapes["bias"]
    return shapes


class GradBuffer:
    """All parameter gradients as views of ONE flat fp32 buffer (one collective per step).

    `alloc(n)` returns a flat 1-D array-like of n fp32 values (numpy.empty, torch.empty on
    a device, ...); views are taken with slicing + reshape, which both libraries return
    as views of a contiguous buffer."""

    def __init__(self, shapes: dict, alloc):
        self.names = [n for n in PARAM_ORDER if n in shapes]
        self.sizes = [int(_prod(shapes[n])) for n in self.names]
        self.numel = sum(self.sizes)
        self.flat = alloc(self.numel)
        self.views = {}
        o = 0
        for n, k in zip(self.names, self.sizes):
            self.views[n] = self.flat[o:o + k].reshape(shapes[n])
            o += k

    def __getitem__(self, name):
        return self.views[name]


def _prod(shape):
    p = 1
    for s in shape:
        p *= int(s)
    return p


def allreduce_torch(flat, group=None):
    """Sum `flat` (a torch tensor) over the ranks of torch.distributed's group."""
    import torch.distributed as dist
    dist.all_reduce(flat, group=group)


class RcclComm:
    """libdcn's RCCL communicator (dcn_comm_init). One per rank; `uid` is the 128-byte id
    made by unique_id() on one rank and shipped to the others by any channel."""

    def __init__(self, handle, nranks: int, rank: int, uid: bytes):
        import dcn_runtime as rt
        if len(uid) != 128:
            raise ValueError("RCCL unique id must be 128 bytes")
        self.handle, self.rt = handle, rt
        self.c = ctypes.c_void_p()
        buf = ctypes.create_string_buffer(uid, 128)
        rt.check(handle.lib.dcn_comm_init(handle.h, nranks, rank, buf, ctypes.byref(self.c)),
                 "dcn_comm_init")

    @staticmethod
    def unique_id() -> bytes:
        import dcn_runtime as rt
        buf = ctypes.create_string_buffer(128)
        rt.check(rt.load().dcn_comm_get_unique_id(buf), "dcn_comm_get_unique_id")
        return buf.raw

    def allreduce(self, dev_ptr: int, count: int, dtype: int = 0):
        """In-place sum of `count` values of `dtype` (dcn_runtime.DCN_F32 / DCN_BF16) at
        device address `dev_ptr`, on the handle's stream. libdcn rejects a count/dtype
        that runs past the allocation holding dev_ptr."""
        self.rt.check(self.handle.lib.dcn_allreduce_grads(self.handle.h, self.c,
                                                          ctypes.c_void_p(dev_ptr), count,
                                                          int(dtype)),
                      "dcn_allreduce_grads")

    def close(self):
        if self.c:
            self.handle.lib.dcn_comm_destroy(self.c)
            self.c = ctypes.c_void_p()
