#!/usr/bin/env python3
"""Probe bf16 GEMM rates (torch -> hipBLASLt / rocBLAS) for the config-4 DeformConv2d GEMM
shapes (B=64, O=256, K=2304, HW=784) in the layouts libdcn could use."""
import time

import torch

B, O, K, HW = 64, 256, 2304, 784
dev = "cuda"
W = torch.randn(O, K, device=dev).bfloat16()
colT = torch.randn(B, HW, K, device=dev).bfloat16()
G = torch.randn(B, O, HW, device=dev).bfloat16()
GT = torch.randn(B * HW, O, device=dev).bfloat16()


def bench(fn, n=20):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / n * 1e3


flop = 2.0 * B * O * K * HW
c2 = colT.view(B * HW, K)
cases = {
    "fwd batched out_b=W@colT_b^T": lambda: torch.matmul(W, colT.transpose(1, 2)),
    "fwd flat outT=colT@W^T [BHW,O]": lambda: torch.matmul(c2, W.t()),
    "dW batched G_b@colT_b": lambda: torch.bmm(G, colT),
    "dW flat GT^T@colT": lambda: torch.matmul(GT.t(), c2),
    "dcol flat GT@W": lambda: torch.matmul(GT, W),
}
for lib in ("cublaslt", "cublas"):
    try:
        torch.backends.cuda.preferred_blas_library(lib)
    except Exception as e:
        print(lib, "unavailable", e)
        continue
    for name, fn in cases.items():
        ms = bench(fn)
        print(f"{lib:9s} {name:34s} {ms * 1e3:8.1f} us  {flop / ms / 1e9:7.1f} TF/s", flush=True)
