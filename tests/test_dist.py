"""Batch-sharded DP on CPU (gloo, world_size 2): per-rank shards through the oracle, the
packed GradBuffer summed with one all_reduce, equal to the single-process full batch —
the same sharding / packing / collective code bench.py runs over RCCL on the GPUs."""
from __future__ import annotations

import os
import socket

import numpy as np
import pytest

import dcn_dp
import dcn_oracle as O
from conftest import assert_close, assert_close_reduction

torch = pytest.importorskip("torch")
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402


def _case(B=5):
    rng = np.random.default_rng(7)
    C, O_, H, W = 6, 5, 9, 8
    x = rng.standard_normal((B, C, H, W)).astype(np.float32)
    wo = (rng.standard_normal((18, C, 3, 3)) / np.sqrt(C * 9)).astype(np.float32)
    bo = rng.uniform(-0.5, 0.5, 18).astype(np.float32)
    w = (rng.standard_normal((O_, C, 3, 3)) * np.sqrt(2 / (C * 9))).astype(np.float32)
    b = (rng.standard_normal(O_) * 0.1).astype(np.float32)
    Ho, Wo = O.out_size(H, W, 3, 3, 1, 1, 1, 1)
    gout = rng.standard_normal((B, O_, Ho, Wo)).astype(np.float32)
    return x, wo, bo, w, b, gout


def _grads(x, wo, bo, w, b, gout):
    _, _, cache = O.forward(x, wo, bo, w, b, (1, 1), (1, 1))
    return O.backward(cache, gout)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, outdir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        x, wo, bo, w, b, gout = _case()
        b0, nb = dcn_dp.shard_range(x.shape[0], world, rank)
        g = _grads(x[b0:b0 + nb], wo, bo, w, b, gout[b0:b0 + nb])
        buf = dcn_dp.GradBuffer(dcn_dp.param_shapes(6, 5, 3, 3),
                                lambda n: torch.empty(n, dtype=torch.float64))
        for name in buf.names:
            buf[name].copy_(torch.from_numpy(np.ascontiguousarray(g[name])))
        dcn_dp.allreduce_torch(buf.flat)
        np.savez(os.path.join(outdir, f"rank{rank}.npz"), flat=buf.flat.numpy(), b0=b0, nb=nb,
                 gx=g["x"], goff=g["offset"])
    finally:
        dist.destroy_process_group()


def test_shard_range_covers_batch():
    for B in (1, 5, 64, 513):
        for world in (1, 2, 3, 8):
            spans = [dcn_dp.shard_range(B, world, r) for r in range(world)]
            assert sum(nb for _, nb in spans) == B
            assert all(spans[i][0] + spans[i][1] == spans[i + 1][0] for i in range(world - 1))
            assert max(nb for _, nb in spans) - min(nb for _, nb in spans) <= 1
    with pytest.raises(ValueError):
        dcn_dp.shard_range(4, 2, 2)


def test_grad_buffer_packing_order():
    shapes = dcn_dp.param_shapes(256, 256, 3, 3)
    buf = dcn_dp.GradBuffer(shapes, lambda n: np.zeros(n, np.float32))
    assert buf.numel == 631_570  # 2.53 MB per step at config 3
    buf["offset_conv.bias"][:] = 1.0
    assert buf.flat[-18:].sum() == 18 and buf.flat[:-18].sum() == 0
    assert "bias" not in dcn_dp.GradBuffer(dcn_dp.param_shapes(4, 4, 3, 3, bias=False),
                                           lambda n: np.zeros(n)).names


def test_two_rank_gloo_allreduce_equals_full_batch(tmp_path):
    world = 2
    mp.start_processes(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world,
                       join=True, start_method="spawn")
    full = _grads(*_case())
    ranks = [np.load(tmp_path / f"rank{r}.npz") for r in range(world)]
    np.testing.assert_array_equal(ranks[0]["flat"], ranks[1]["flat"])  # replicas agree
    buf = dcn_dp.GradBuffer(dcn_dp.param_shapes(6, 5, 3, 3), lambda n: ranks[0]["flat"])
    for name in buf.names:
        assert_close_reduction(buf[name], full[name], what=f"dp {name}")
    for z in ranks:  # per-image grads need no exchange
        b0, nb = int(z["b0"]), int(z["nb"])
        assert_close(z["gx"], full["x"][b0:b0 + nb], what="dp ∂x shard")
        assert_close(z["goff"], full["offset"][b0:b0 + nb], what="dp ∂offset shard")
