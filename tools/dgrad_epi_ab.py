#!/usr/bin/env python3
"""A/B: short-K pointwise data gradients with the accumulate + BN-statistics epilogue (the c1
dgrads of ResNet-50 stages 2-5 at b1024) on the 256-row kernel vs the 4-wave kernel (two
workgroups per CU: one's epilogue overlaps the other's main loop). usage: python tools/dgrad_epi_ab.py"""
import statistics
import sys

import torch

sys.path.insert(0, ".")
from tensorflow_train_distributed_amd.ops import gemm as G  # noqa: E402

B = 1024
# (name, H, C = dx channels, K = dz channels)
SHAPES = [("s2 c1", 56, 256, 64), ("s3 c1", 28, 512, 128), ("s4 c1", 14, 1024, 256), ("s5 c1", 7, 2048, 512),
          ("s3 c3", 28, 128, 512), ("s4 c3", 14, 256, 1024)]


def timeit(fn, n=5):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n * 1e3


for name, H, C, K in SHAPES:
    M = B * H * H
    dz = torch.randn(B, H, H, K, device="cuda").bfloat16()
    wt = (torch.randn(C, 1, 1, K, device="cuda") / K ** 0.5).bfloat16()
    y = torch.randn(B, H, H, C, device="cuda").bfloat16()
    bits = torch.randint(0, 256, (M * C // 8,), dtype=torch.uint8, device="cuda")
    dx = torch.randn(B, H, H, C, device="cuda").bfloat16()
    res = {}
    outs = {}
    for mode, lim in (("big256", 0), ("4wave", 1 << 20)):
        G.DGRAD_STAT_4W_K = lim
        fn = lambda: G.conv_dgrad(dz, wt, (B, H, H, C), out=dx, beta=1, bn_stat=(y, bits))  # noqa: E731
        fn()
        torch.cuda.synchronize()
        res[mode] = [timeit(fn) for _ in range(3)]
        d0 = dx.clone()
        o = G.conv_dgrad(dz, wt, (B, H, H, C), out=d0, beta=0, bn_stat=(y, bits))
        outs[mode] = (o[0].float(), o[1][: o[2]].sum(0))
    G.DGRAD_STAT_4W_K = 0
    err = float((outs["big256"][0] - outs["4wave"][0]).abs().max())
    serr = float(((outs["big256"][1] - outs["4wave"][1]).abs() / (outs["big256"][1].abs() + 1)).max())
    byt = 2 * (M * K + 3 * M * C) + M * C // 8
    print("%-6s M=%-7d C=%-5d K=%-4d " % (name, M, C, K) + "  ".join(
        "%s %6.1f us (%.2f TB/s)" % (k, statistics.median(v), byt / statistics.median(v) / 1e6) for k, v in res.items())
        + "  | out maxdiff %.3g stat reldiff %.3g" % (err, serr), flush=True)
