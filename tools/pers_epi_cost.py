#!/usr/bin/env python3
"""Cost of the persistent 256-row GEMM's epilogue kinds on BERT-Large b128 shapes (M = 65536
tokens): plain store vs bias vs bias+GELU+aux vs dGELU (reads the pre-activation) vs beta
(reads the output). usage: python tools/pers_epi_cost.py"""
import sys

import torch

sys.path.insert(0, ".")
from tensorflow_train_distributed_amd.ops import gemm as G  # noqa: E402


def timeit(fn, iters=10):
    for _ in range(2):
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
for name, M, N, K in (("ffn1/ffn2-dgrad", T, 4096, 1024), ("qkv", T, 3072, 1024), ("proj/ffn2", T, 1024, 4096)):
    a = (torch.rand(M, K, device="cuda") * 2 - 1).bfloat16()
    b = (torch.rand(N, K, device="cuda") * 2 - 1).bfloat16()
    bias = torch.randn(N, device="cuda")
    pre = torch.randn(M, N, device="cuda").bfloat16()
    out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    aux = torch.empty_like(out)
    fl = 2.0 * M * N * K
    r = {
        "plain": timeit(lambda: G.gemm(a, b, trans_b=True, out=out)),
        "bias": timeit(lambda: G.gemm(a, b, trans_b=True, out=out, bias=bias)),
        "gelu+aux": timeit(lambda: G.gemm(a, b, trans_b=True, out=out, bias=bias, act=G.ACT_GELU, aux=aux)),
        "dgelu": timeit(lambda: G.gemm(a, b, trans_b=True, out=out, act=G.ACT_DGELU, residual=pre)),
        "beta": timeit(lambda: G.gemm(a, b, trans_b=True, out=out, beta=1)),
    }
    print("%-16s M=%d N=%d K=%d  " % (name, M, N, K) + "  ".join(
        "%s %6.1f us (%4.0f TF/s)" % (k, v, fl / v / 1e6) for k, v in r.items()), flush=True)
    del a, b, pre, out, aux
