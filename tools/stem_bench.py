#!/usr/bin/env python3
"""Stem weight gradient at batch B: dedicated kernel (stem_wgrad.hip) vs the generic
im2col-gather GEMM with the BN backward on load (conv_wgrad_bn). usage: stem_bench.py [B]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from tensorflow_train_distributed_amd.ops import gemm as G  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
x = torch.zeros(B, 224, 224, 8, device="cuda", dtype=torch.bfloat16)
x[..., :3] = torch.randn(B, 224, 224, 3, device="cuda").bfloat16()
g = torch.randn(B, 112, 112, 64, device="cuda").bfloat16()
y = torch.randn(B, 112, 112, 64, device="cuda").bfloat16()
coef = torch.randn(3, 64, device="cuda") * 0.1
out = torch.empty(64, 7, 7, 8, device="cuda")


def timeit(fn, n=5):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n * 1e3


t_new = timeit(lambda: G.stem_wgrad(x, g, y, coef, out=out))
t_old = timeit(lambda: G.conv_wgrad_bn(x, g, y, coef, (64, 7, 7, 8), (2, 2), (3, 3), out=out))
x3 = x[..., :3].contiguous()
t3 = timeit(lambda: G.stem_wgrad(x3, g, y, coef, out=out))
gb = (g.numel() * 2 * 2 + x.numel() * 2) / 1e9
print("stem wgrad b%d, packed RGB input (the ResNet step's): %.1f us" % (B, t3), flush=True)
print("stem wgrad b%d: kernel %.1f us (%.2f TB/s of g+y+x)  generic %.1f us" % (B, t_new, gb / t_new * 1e3, t_old),
      flush=True)

