#!/usr/bin/env python3
"""Split-K sweep of the 4-wave weight-gradient kernels (small M x N, K = pixels) at ResNet-50
b1024 shapes: the wgrad_splits() default vs 2x / 3x / 4x. usage: python tools/wgrad_split_sweep.py"""
import sys

import torch

sys.path.insert(0, ".")
from tensorflow_train_distributed_amd.ops import gemm as G  # noqa: E402

B = 1024
LAYERS = [  # name, H(in), Cin, Cout, k, stride, pad
    ("stem7x7", 224, 8, 64, 7, 2, 3),
    ("s1_3x3", 56, 64, 64, 3, 1, 1),
    ("s1_1x1_256to64", 56, 256, 64, 1, 1, 0),
    ("s1_1x1_64to256", 56, 64, 256, 1, 1, 0),
    ("s1_1x1_64to64", 56, 64, 64, 1, 1, 0),
    ("s2_3x3", 28, 128, 128, 3, 1, 1),
]


def timeit(f, n=5):
    for _ in range(2):
        f()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n):
        f()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n * 1e3


for name, H, C, K, k, st, p in LAYERS:
    x = torch.randn(B, H, H, C, device="cuda").bfloat16()
    P = (H + 2 * p - k) // st + 1
    dy = torch.randn(B, P, P, K, device="cuda").bfloat16()
    ws = (K, k, k, C)
    g = G.conv_geom(x.shape, ws, (st, st), (p, p))
    base = G.wgrad_splits(g)
    res = []
    for mul in (1, 2, 3, 4):
        sp = base * mul
        t = timeit(lambda: G.conv_wgrad(x, dy, ws, (st, st), (p, p), splits=sp))
        res.append("x%d(%d) %7.1f" % (mul, sp, t))
    print("%-16s " % name + "  ".join(res), flush=True)
    del x, dy
