#!/usr/bin/env python3
"""Run BERT's weight-gradient GEMM (dW = dy^T . x with the fused bias row sums, split-K as the
BERT engine sizes it) repeatedly, for rocprofv3 --pmc passes / timing.
usage: one_wgrad.py M N K [iters] [wgs]    (dW [M, N], K tokens; wgs = workgroup target, 192)"""
import sys
import time

import torch

sys.path.insert(0, ".")
from tensorflow_train_distributed_amd.ops import gemm as G  # noqa: E402

M, N, K = (int(v) for v in sys.argv[1:4])
iters = int(sys.argv[4]) if len(sys.argv) > 4 else 10
wgs = int(sys.argv[5]) if len(sys.argv) > 5 else 192
dy = (torch.rand((K, M), device="cuda") * 2 - 1).bfloat16()
x = (torch.rand((K, N), device="cuda") * 2 - 1).bfloat16()
w = torch.empty((M, N), dtype=torch.float32, device="cuda")
b = torch.empty((M,), dtype=torch.float32, device="cuda")
splits = G.gemm_wgrad_splits(M, N, K, big_wgs=wgs)
for _ in range(3):
    G.gemm_wgrad_bias(dy, x, w, b, splits=splits)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(iters):
    G.gemm_wgrad_bias(dy, x, w, b, splits=splits)
torch.cuda.synchronize()
dt = (time.perf_counter() - t0) / iters
print("wgrad M=%d N=%d K=%d splits=%d: %.1f us  %.0f TF/s" % (M, N, K, splits, dt * 1e6, 2.0 * M * N * K / dt / 1e12))
