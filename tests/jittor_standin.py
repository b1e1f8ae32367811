"""A minimal stand-in for the parts of Jittor that jittor-dcn_amd/deform_conv.py's Jittor
backend touches — TEST INFRASTRUCTURE ONLY (Jittor itself is not installable here, SURVEY
§8(c)). It restates the protocol, not Jittor's implementation:

* `jt.Function.apply(*args)` runs `execute(*args)`; inputs that are Vars are recorded in an
  input mask, everything else (None bias, stride / padding tuples) is not. The backward
  calls `grad(*grad_outputs)`, which must return ONE entry per input, in input order,
  and `None` for every non-Var input — the contract Jittor's Function enforces in its
  `_grad` (an assertion that the i-th returned grad is None when input i is not a Var).
* `Var` wraps a NumPy array (`.numpy()`, `.shape`); `jt.array` makes one.
* `jt.nn.Module`, `jt.nn.Conv` (weight [out, in, kh, kw], bias [out]), `jt.init.gauss`,
  `jt.init.constant`, `jt.zeros_like` — what DeformConv2d's constructor uses
  (deform_conv.py:16-28 of the reference).

`install()` puts it into sys.modules as `jittor` / `jittor.nn` and returns it.
"""
from __future__ import annotations

import sys
import types

import numpy as np


class Var:
    def __init__(self, a):
        self._a = np.array(a, np.float32)

    def numpy(self):
        return self._a

    @property
    def shape(self):
        return self._a.shape

    def is_stop_grad(self):
        return False


def array(a):
    return Var(a)


def zeros_like(v):
    return Var(np.zeros_like(v.numpy()))


class Module:
    def __call__(self, *args, **kw):
        return self.execute(*args, **kw)

    def parameters(self):
        out = []
        for v in vars(self).values():
            if isinstance(v, Var):
                out.append(v)
            elif isinstance(v, Module):
                out.extend(v.parameters())
        return out


class Function(Module):
    """apply -> execute, with the input mask Jittor's Function keeps; the last applied
    instance is kept in `Function.last` so a test can run its backward."""

    last = None

    @classmethod
    def apply(cls, *args):
        f = cls()
        f.input_mask = [isinstance(a, Var) for a in args]
        Function.last = f
        return f.execute(*args)

    def backward(self, *grad_outputs):
        """Jittor's _grad: one returned grad per input; non-Var inputs must get None.
        Returns the grads of the Var inputs, in input order."""
        ret = self.grad(*grad_outputs)
        if not isinstance(ret, (tuple, list)):
            ret = (ret,)
        if len(ret) != len(self.input_mask):
            raise AssertionError(f"{type(self).__name__}.grad returned {len(ret)} grads for "
                                 f"{len(self.input_mask)} inputs")
        out = []
        for i, (r, is_var) in enumerate(zip(ret, self.input_mask)):
            if not is_var:
                assert r is None, (f"{type(self).__name__}'s {i}-th returned grad should be "
                                   "None, because the input value is not jittor variable.")
            else:
                out.append(r)
        return out


class Conv(Module):
    def __init__(self, in_channels, out_channels, kernel_size, stride=1, padding=0):
        kh, kw = kernel_size if isinstance(kernel_size, tuple) else (kernel_size,) * 2
        rng = np.random.default_rng(0)
        self.weight = Var(rng.standard_normal((out_channels, in_channels, kh, kw)))
        self.bias = Var(rng.standard_normal(out_channels))
        self.stride, self.padding = stride, padding


def _gauss(shape, mean=0.0, std=1.0):
    return Var(np.random.default_rng(1).normal(mean, std, shape))


def _constant(shape, value=0.0):
    return Var(np.full(shape, value, np.float32))


def install():
    jt = types.ModuleType("jittor")
    jt.Var, jt.array, jt.zeros_like, jt.Function, jt.Module = Var, array, zeros_like, Function, \
        Module
    nn = types.ModuleType("jittor.nn")
    nn.Module, nn.Conv = Module, Conv
    jt.nn = nn
    jt.init = types.SimpleNamespace(gauss=_gauss, constant=_constant)
    sys.modules["jittor"] = jt
    sys.modules["jittor.nn"] = nn
    return jt


def uninstall():
    sys.modules.pop("jittor", None)
    sys.modules.pop("jittor.nn", None)
