#!/usr/bin/env python3
"""What the accumulate (beta) epilogue costs the 4-wave GEMM at BERT-Large data-gradient shapes:
the same GEMM with beta = 0 and beta = 1 (C += A . B^T), HIP-event timed.
usage: python tools/g4_beta_bench.py"""
import sys

import torch

sys.path.insert(0, ".")
from tensorflow_train_distributed_amd.ops import gemm as G  # noqa: E402


def timeit(fn, iters=10):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


T = 65536
for name, M, N, K in (("ao_dgrad", T, 1024, 1024), ("qkv_dgrad", T, 1024, 3072), ("ffn1_dgrad", T, 1024, 4096)):
    a = (torch.rand((M, K), device="cuda") * 2 - 1).bfloat16()
    b = (torch.rand((N, K), device="cuda") * 2 - 1).bfloat16()
    out = torch.zeros(M, N, device="cuda", dtype=torch.bfloat16)
    t0 = timeit(lambda: G.gemm4w(a, b, out=out))
    t1 = timeit(lambda: G.gemm4w(a, b, out=out, beta=1))
    fl = 2.0 * M * N * K
    print("%-11s %6d x %5d x %5d  beta0 %7.1f us %5.0f TF/s   beta1 %7.1f us %5.0f TF/s"
          % (name, M, N, K, t0, fl / t0 / 1e6, t1, fl / t1 / 1e6))
