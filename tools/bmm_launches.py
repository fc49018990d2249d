#!/usr/bin/env python3
"""Batched MatMul launch count (ops.gemm.gemm_batched via nn MatMul): run under rocprofv3
--kernel-trace; every call must be ONE GEMM kernel dispatch (batch index on the grid)."""
import sys

import torch

sys.path.insert(0, ".")
from tensorflow_train_distributed_amd.ops import gemm as G  # noqa: E402

for (bt, m, k, n) in [(8, 512, 64, 512), (16, 512, 512, 64)]:
    a = torch.randn(bt, m, k, device="cuda").bfloat16()
    b = torch.randn(bt, k, n, device="cuda").bfloat16()
    torch.cuda.synchronize()
    for _ in range(5):
        G.gemm_batched(a, b)
    torch.cuda.synchronize()
print("calls: 10")
