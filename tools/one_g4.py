#!/usr/bin/env python3
"""One GEMM shape on the 4-wave kernel (or torch.mm), for rocprofv3 passes.
usage: one_g4.py M N K [sched (1 | 0 | torch)] [iters]"""
import sys

import torch

sys.path.insert(0, ".")
from tensorflow_train_distributed_amd.ops import gemm as G  # noqa: E402

M, N, K = (int(x) for x in sys.argv[1:4])
mode = sys.argv[4] if len(sys.argv) > 4 else "1"
iters = int(sys.argv[5]) if len(sys.argv) > 5 else 10
a = (torch.rand((M, K), device="cuda") * 2 - 1).bfloat16()
b = (torch.rand((N, K), device="cuda") * 2 - 1).bfloat16()
out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
if mode != "torch":
    G.set_g4_sched(int(mode))
for _ in range(iters):
    if mode == "torch":
        torch.mm(a, b.t(), out=out)
    else:
        G.gemm4w(a, b, out=out)
torch.cuda.synchronize()
