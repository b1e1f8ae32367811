#!/usr/bin/env python3
"""fp32 GEMM throughput, batched-per-image vs flattened over the batch (B*HW rows), for
the three DeformConv2d GEMMs at config 3, through torch (rocBLAS / hipBLASLt)."""
import time

import torch

B, O, K, HW = 64, 256, 2304, 3136
dev = "cuda"
W = torch.randn(O, K, device=dev)
colT = torch.randn(B, HW, K, device=dev)
G = torch.randn(B, O, HW, device=dev)
GT = torch.randn(B * HW, O, device=dev)
cf = colT.view(B * HW, K)


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
    "fwd  batched": lambda: torch.matmul(W, colT.transpose(1, 2)),
    "fwd  flat outT=cf@W^T": lambda: torch.matmul(cf, W.t()),
    "dW   batched": lambda: torch.bmm(G, colT),
    "dW   flat GT^T@cf": lambda: torch.matmul(GT.t(), cf),
    "dW   flat cf^T@GT": lambda: torch.matmul(cf.t(), GT),
    "dcol batched": lambda: torch.matmul(G.transpose(1, 2), W),
    "dcol flat GT@W": lambda: torch.matmul(GT, W),
}
for lib in ("cublas", "cublaslt"):
    try:
        torch.backends.cuda.preferred_blas_library(lib)
    except Exception as e:
        print(lib, "unavailable", e)
        continue
    for name, fn in cases.items():
        ms = bench(fn)
        print(f"{lib:9s} {name:24s} {ms:7.3f} ms  {flop / ms / 1e9:7.1f} TF/s", flush=True)
x = torch.randn(B, O, HW, device=dev)
ms = bench(lambda: x.transpose(1, 2).contiguous())
print(f"transpose [B,O,HW]->[B,HW,O] {ms:.3f} ms")
