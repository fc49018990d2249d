#!/usr/bin/env python3
"""Run one dense GEMM repeatedly (rocprofv3 --pmc passes / timing).
usage: one_gemm.py M N K [ta tb iters tile]"""
import sys
import time

import torch

sys.path.insert(0, ".")
from tensorflow_train_distributed_amd.ops import gemm as G  # noqa: E402

M, N, K = (int(v) for v in sys.argv[1:4])
ta = len(sys.argv) > 4 and sys.argv[4] == "1"
tb = len(sys.argv) > 5 and sys.argv[5] == "1"
iters = int(sys.argv[6]) if len(sys.argv) > 6 else 20
tile = int(sys.argv[7]) if len(sys.argv) > 7 else 256
a = (torch.rand((K, M) if ta else (M, K), device="cuda") * 2 - 1).bfloat16()
b = (torch.rand((N, K) if tb else (K, N), device="cuda") * 2 - 1).bfloat16()
out = torch.empty((M, N), dtype=torch.bfloat16, device="cuda")
for _ in range(3):
    G.gemm(a, b, trans_a=ta, trans_b=tb, out=out, tile=(tile, tile))
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(iters):
    G.gemm(a, b, trans_a=ta, trans_b=tb, out=out, tile=(tile, tile))
torch.cuda.synchronize()
dt = (time.perf_counter() - t0) / iters
print("M=%d N=%d K=%d ta=%d tb=%d: %.1f us  %.0f TF/s" % (M, N, K, ta, tb, dt * 1e6, 2.0 * M * N * K / dt / 1e12))
