"""CPU: the drop-in module surface of deform_conv.DeformConv2d (deform_conv.py:6-28)
and the reference's call protocol (train.py:311-320, :351, :461; test.py:19)."""
import math
import os

import numpy as np
import pytest

import deform_conv
import dcn_runtime as rt
from deform_conv import DeformConv2d, dcn_backward_numpy, dcn_forward_numpy


def test_import_line_matches_reference():
    # train.py:299 / test.py:12: `from deform_conv import DeformConv2d`
    assert DeformConv2d.__name__ in ("DeformConv2d", "DeformConv2dNumpy")
    assert not deform_conv.HAVE_JITTOR or DeformConv2d.__name__ == "DeformConv2d"


def test_constructor_defaults_and_tuples():
    m = DeformConv2d(16, 32)
    assert (m.in_channels, m.out_channels) == (16, 32)
    assert m.kernel_size == (3, 3) and m.stride == (1, 1) and m.padding == (1, 1)
    assert m.N == 9
    m2 = DeformConv2d(16, 32, 3, 2, 1)  # positional, as train.py:311
    assert m2.stride == (2, 2)
    m3 = DeformConv2d(4, 8, (3, 2), (1, 2), (1, 0), bias=False)
    assert m3.kernel_size == (3, 2) and m3.N == 6 and m3.bias is None


def test_parameters_shapes_and_init():
    m = DeformConv2d(64, 128, 3, 2, 1)
    assert m.offset_conv.weight.shape == (18, 64, 3, 3)
    assert m.offset_conv.bias.shape == (18,)
    assert m.weight.shape == (128, 64, 3, 3)
    assert m.bias.shape == (128,)
    # zero offset-conv init (deform_conv.py:27-28), zero bias (:25)
    assert not np.any(m.offset_conv.weight) and not np.any(m.offset_conv.bias)
    assert not np.any(m.bias)
    # He-normal weight std (deform_conv.py:23)
    assert abs(np.std(m.weight) - math.sqrt(2.0 / (64 * 9))) < 0.05 * math.sqrt(2.0 / (64 * 9))
    assert all(p.dtype == np.float32 for p in m.parameters())


def test_state_dict_keys_round_trip(tmp_path):
    m = DeformConv2d(4, 6)
    keys = set(m.state_dict())
    assert keys == {"weight", "bias", "offset_conv.weight", "offset_conv.bias"}
    path = os.path.join(tmp_path, "sd.npz")
    m.save(path)
    m2 = DeformConv2d(4, 6, seed=123)
    m2.load(path)
    for k, v in m.state_dict().items():
        np.testing.assert_array_equal(m2.state_dict()[k], v)
    with pytest.raises(ValueError):
        DeformConv2d(5, 6).load_state_dict(m.state_dict())


def test_parameters_feed_an_optimizer():
    m = DeformConv2d(4, 6)
    assert len(m.parameters()) == 4
    m.zero_grad()
    assert all(p.grad is None for p in m.parameters())


def test_execute_without_gpu_fails_loudly():
    if rt.device_count() > 0:
        pytest.skip("a HIP device is visible")
    m = DeformConv2d(2, 3)
    with pytest.raises(RuntimeError):
        m(np.zeros((1, 2, 8, 8), np.float32))


def test_empty_batch_through_the_module():
    """B == 0: execute + backward through the module give empty outputs and zero
    parameter grads without a launch (so without a device), as the reference's ops do on an
    empty batch; the forward-reuse context is None and the backward accepts it."""
    m = DeformConv2d(3, 5, 3, 2, 1)
    x = np.zeros((0, 3, 9, 7), np.float32)
    out = m(x)
    assert out.shape == (0, 5, 5, 4) and out.dtype == np.float32
    gx = m.backward(np.zeros_like(out))
    assert gx.shape == x.shape
    for name, p in m.named_parameters():
        assert p.grad.shape == p.shape and not p.grad.any(), name
    # the functional form, with and without the context
    o2, off, ctx = dcn_forward_numpy(x, m.offset_conv.weight, m.offset_conv.bias, m.weight, None,
                                     (2, 2), (1, 1), return_ctx=True)
    assert ctx is None and o2.shape == (0, 5, 5, 4) and off.shape == (0, 18, 5, 4)
    g = dcn_backward_numpy(x, off, m.offset_conv.weight, m.weight, False, o2, (2, 2), (1, 1),
                           ctx=ctx)
    assert "bias" not in g and g["offset"].shape == off.shape
