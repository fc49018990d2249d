#!/usr/bin/env python3
"""One weight-gradient shape on the 4-wave transposed-read kernel (or torch.mm), for rocprofv3
passes. usage: one_g4t.py M N K [splits | torch] [iters] [bias]"""
import sys

import torch

sys.path.insert(0, ".")
from tensorflow_train_distributed_amd.ops import gemm as G  # noqa: E402

M, N, K = (int(x) for x in sys.argv[1:4])
mode = sys.argv[4] if len(sys.argv) > 4 else "4"
iters = int(sys.argv[5]) if len(sys.argv) > 5 else 10
dy = (torch.rand((K, M), device="cuda") * 2 - 1).bfloat16()
x = (torch.rand((K, N), device="cuda") * 2 - 1).bfloat16()
out = torch.empty(M, N, device="cuda")
bias = torch.empty(M, device="cuda") if len(sys.argv) > 6 else None
for _ in range(iters):
    if mode == "torch":
        torch.mm(dy.t(), x, out_dtype=torch.float32, out=out)
    else:
        G.gemm4t(dy, x, out, bias, splits=int(mode))
torch.cuda.synchronize()
