#!/usr/bin/env python3
"""Time the fused attention kernels at BERT-Large shapes (B=32, H=16, S=512, D=64) with and
without attention dropout; the backward on the single-kernel path and on the split dQ / dK-dV
kernels. usage: python tools/attn_bench.py [B]"""
import sys

import torch

sys.path.insert(0, ".")
from tensorflow_train_distributed_amd.ops import transformer as T  # noqa: E402


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


B, H, S, D = (int(sys.argv[1]) if len(sys.argv) > 1 else 32), 16, 512, 64
qkv = (torch.randn(B * S, 3 * H * D, device="cuda") * 0.5).bfloat16()
q, k, v = qkv[:, :H * D], qkv[:, H * D:2 * H * D], qkv[:, 2 * H * D:]
out = torch.empty(B * S, H * D, device="cuda", dtype=torch.bfloat16)
lse = torch.empty(B * H, S, device="cuda")
dout = torch.randn_like(out)
dqkv = torch.empty_like(qkv)
rng = T.RngState(7, "cuda")
fl_f = 4.0 * B * H * S * S * D
for p in (0.0, 0.1):
    tf = timeit(lambda: T.attention_fwd(q, k, v, out, lse, B, H, S, p_drop=p, rng=rng))
    res = {}
    for fused in (True, False):
        T.set_fused_attention_bwd(fused)
        res[fused] = timeit(lambda: T.attention_bwd(q, k, v, out, dout, lse, dqkv[:, :H * D], dqkv[:, H * D:2 * H * D],
                                                    dqkv[:, 2 * H * D:], B, H, S, p_drop=p, rng=rng))
    T.set_fused_attention_bwd(False)
    # backward FLOPs counted as the algorithm's 5 products (2.5x the forward's 2)
    print("p=%.1f  fwd %6.1f us %5.0f TF/s   bwd fused %6.1f us %5.0f TF/s   split %6.1f us %5.0f TF/s"
          % (p, tf, fl_f / tf / 1e6, res[True], 2.5 * fl_f / res[True] / 1e6, res[False], 2.5 * fl_f / res[False] / 1e6))
