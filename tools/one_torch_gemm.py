#!/usr/bin/env python3
"""Run one torch.matmul (hipBLASLt) GEMM repeatedly, for PMC comparisons with tools/one_gemm.py.
usage: one_torch_gemm.py M N K [iters]"""
import sys

import torch

M, N, K = (int(v) for v in sys.argv[1:4])
iters = int(sys.argv[4]) if len(sys.argv) > 4 else 10
a = (torch.rand((M, K), device="cuda") * 2 - 1).bfloat16()
b = (torch.rand((N, K), device="cuda") * 2 - 1).bfloat16()
for _ in range(iters + 3):
    torch.matmul(a, b.t())
torch.cuda.synchronize()
print("done")
