"""Split-bf16 fp32 GEMM (csrc/dcn_gemm_split.hip, DCN_MATH_F32_BF16X*) against float64.

Every fp32 operand is split exactly into bf16 planes and the plane products run on the
bf16 matrix cores with fp32 accumulation. The bar for X9 and X6 is native-f32 accuracy:
their error against a float64 product of the same fp32 operands must stay within a small
factor of the native f32 MFMA GEMM's own error (vendor libraries, DCN_MATH_F32). X3 is
the opt-in two-plane mode (~2^-17 relative per product).
"""
import ctypes

import numpy as np
import pytest

import dcn_runtime as rt
from test_gpu_parity import Dev, _check, _device_fwd_bwd, _oracle, _rand_case

pytestmark = pytest.mark.gpu

# (ta, tb, m, n, k, batch): every operand layout, ragged tiles (m, n not multiples of 128;
# k not a multiple of 32), the three config-3 layouts in miniature
CASES = [
    (True, False, 196, 136, 100, 2),    # forward: out = colᵀ·W (both k-contiguous)
    (False, False, 200, 72, 148, 3),    # ∂W per image: A m-contiguous, B k-contiguous
    (False, True, 132, 260, 64, 1),     # per-image ∂col NT: B n-contiguous
    (True, True, 64, 68, 36, 2),        # both transposed
    (False, False, 576, 784, 256, 1),   # ∂col flat (k = O = 256)
]


def _run(h, math, ta, tb, m, n, k, batch, A, B):
    D = Dev(h)
    try:
        pa, pb = D.up(A), D.up(B)
        lda = k if ta else m
        ldb = n if tb else k
        pc = D.zeros(batch * m * n * 4)
        h.set_math(math)
        rt.check(h.lib.dcn_debug_gemm(h.h, int(ta), int(tb), m, n, k, ctypes.c_void_p(pa), lda,
                                      A[0].size if batch > 1 else 0, ctypes.c_void_p(pb), ldb,
                                      B[0].size if batch > 1 else 0, ctypes.c_void_p(pc), m,
                                      m * n, batch), "dcn_debug_gemm")
        # C stored column-major per batch: C[b][j][i]
        return D.down(pc, (batch, n, m))
    finally:
        h.set_math(0)
        D.free()


@pytest.mark.parametrize("case", CASES)
def test_split_gemm_accuracy(gpu_handle, case):
    ta, tb, m, n, k, batch = case
    rng = np.random.default_rng(m * 7 + n)
    # column-major storage as row-major arrays: A is (k if ta) [m][k] else [k][m]
    A = rng.standard_normal((batch, m, k) if ta else (batch, k, m)).astype(np.float32)
    B = rng.standard_normal((batch, n, k) if not tb else (batch, k, n)).astype(np.float32)
    # op(B)(kk, j): !tb → B[kk + j·ldb] = row-major [n][k]; tb → [k][n]
    opB = np.swapaxes(B.astype(np.float64), 1, 2) if not tb else B.astype(np.float64)
    opA = A.astype(np.float64) if ta else np.swapaxes(A.astype(np.float64), 1, 2)
    ref = np.einsum("bmk,bkn->bnm", opA, opB)
    scale = np.einsum("bmk,bkn->bnm", np.abs(opA), np.abs(opB))  # Σ|a·b|
    native = _run(gpu_handle, 0, ta, tb, m, n, k, batch, A, B)
    e_native = np.max(np.abs(native - ref) / scale)
    assert e_native < 1e-6, f"native f32 GEMM error {e_native:.2e}"
    for math, bound in ((9, max(3 * e_native, 2e-7)), (6, max(4 * e_native, 3e-7)),
                        (3, 3e-5)):
        got = _run(gpu_handle, math, ta, tb, m, n, k, batch, A, B)
        e = np.max(np.abs(got - ref) / scale)
        assert e <= bound, f"X{math}: max|Δ|/Σ|ab| = {e:.2e} > {bound:.2e} (native {e_native:.2e})"


def test_split_gemm_exact_on_integer_data(gpu_handle):
    """Small integers split into the hi plane alone, so every mode is exact: catches any
    fragment / layout mix-up (asymmetric operands, ragged edges) independent of rounding."""
    rng = np.random.default_rng(5)
    for ta, tb, m, n, k, batch in CASES:
        A = rng.integers(-8, 9, (batch, m, k) if ta else (batch, k, m)).astype(np.float32)
        B = rng.integers(-8, 9, (batch, n, k) if not tb else (batch, k, n)).astype(np.float32)
        opA = A.astype(np.float64) if ta else np.swapaxes(A.astype(np.float64), 1, 2)
        opB = np.swapaxes(B.astype(np.float64), 1, 2) if not tb else B.astype(np.float64)
        ref = np.einsum("bmk,bkn->bnm", opA, opB)
        for math in (3, 6, 9):
            got = _run(gpu_handle, math, ta, tb, m, n, k, batch, A, B)
            np.testing.assert_array_equal(got, ref, err_msg=f"X{math} {(ta, tb, m, n, k, batch)}")


def test_math_mode_roundtrip(gpu_handle):
    for m in (0, 3, 6, 9):
        gpu_handle.set_math(m)
        assert gpu_handle.get_math() == m
    gpu_handle.set_math(0)
    with pytest.raises(RuntimeError):
        gpu_handle.set_math(5)


@pytest.mark.parametrize("math", [6, 9])
@pytest.mark.parametrize("case", [
    # the split kernels stage float4s: a GEMM whose contiguous extent is not a multiple of
    # 4 (the last case's per-image ∂W, k = Ho·Wo = 90) takes the vendor-f32 route instead
    dict(seed=1, B=2, C=32, O_=24, H=28, W=28),
    dict(seed=2, B=3, C=16, O_=16, H=24, W=24, s=(2, 2)),
    dict(seed=7, B=2, C=320, O_=16, H=8, W=10),
    dict(seed=9, B=2, C=64, O_=128, H=32, W=30),
    dict(seed=10, B=2, C=16, O_=8, H=9, W=10),
])
def test_dcn_under_split_math_vs_oracle(gpu_handle, math, case):
    """The whole op (forward + backward) with its three GEMMs in split-bf16 arithmetic
    meets the same north-star tolerance as native f32 against the oracle."""
    c = _rand_case(**case)
    gpu_handle.set_math(math)
    try:
        out, off, g = _device_fwd_bwd(gpu_handle, c)
    finally:
        gpu_handle.set_math(0)
    ro, roff, rg = _oracle(c, off)
    _check(out, off, g, ro, roff, rg, c["b"] is not None, f"X{math} {case}")
