#!/usr/bin/env python3
"""Probe fp32 GEMM throughput of rocBLAS vs hipBLASLt (through torch) for the three
DeformConv2d GEMM shapes at config 3 (B=64, O=256, K=2304, HW=3136)."""
import time

import torch

B, O, K, HW = 64, 256, 2304, 3136
dev = "cuda"
W = torch.randn(O, K, device=dev)
colT = torch.randn(B, HW, K, device=dev)
G = torch.randn(B, O, HW, device=dev)


def bench(fn, n=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / n * 1e3


flop = 2.0 * B * O * K * HW
cases = {
    "fwd  out=W@colT^T": lambda: torch.matmul(W, colT.transpose(1, 2)),
    "dW   G@colT": lambda: torch.bmm(G, colT),
    "dcol G^T@W": lambda: torch.matmul(G.transpose(1, 2), W),
}
for lib in ("cublas", "cublaslt"):
    try:
        torch.backends.cuda.preferred_blas_library(lib)
    except Exception as e:
        print(lib, "unavailable", e)
        continue
    for name, fn in cases.items():
        ms = bench(fn)
        print(f"{lib:9s} {name:20s} {ms:7.3f} ms  {flop / ms / 1e9:7.1f} TF/s")
Wb, cb = W.bfloat16(), colT.bfloat16()
ms = bench(lambda: torch.matmul(Wb, cb.transpose(1, 2)))
print(f"bf16 fwd {ms:.3f} ms {flop / ms / 1e9:.1f} TF/s")
