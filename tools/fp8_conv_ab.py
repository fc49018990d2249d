#!/usr/bin/env python3
"""bf16 vs fp8 (e4m3) forward convs (8-wave conv_fwd_fp8 and the 4-wave conv_fwd4k8) at ResNet-50 b1024 shapes, with the BN-statistics
epilogue as the engine runs them. usage: python tools/fp8_conv_ab.py"""
import sys

import torch

sys.path.insert(0, ".")
from tensorflow_train_distributed_amd.ops import gemm as G  # noqa: E402
from tensorflow_train_distributed_amd.ops import kernels as K  # noqa: E402


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


N = 1024
shapes = [  # (H, Cin, Cout, k, stride)
    (56, 256, 64, 1, 1), (56, 64, 256, 1, 1), (28, 128, 512, 1, 1), (28, 512, 128, 1, 1), (28, 128, 128, 3, 1),
    (14, 256, 1024, 1, 1), (14, 1024, 256, 1, 1), (14, 256, 256, 3, 1), (7, 512, 2048, 1, 1), (7, 512, 512, 3, 1),
]
for H, C, Ko, k, s in shapes:
    x = torch.randn(N, H, H, C, device="cuda").bfloat16()
    w = (torch.randn(Ko, k, k, C, device="cuda") / (k * k * C) ** 0.5).bfloat16()
    pad = k // 2
    P = (H + 2 * pad - k) // s + 1
    M = N * P * P
    big = G.big_bn(M, Ko, k * k * C)  # the engine's tile choice (models/resnet.py _convbn_fwd)
    tile = (256, big) if big and C % 64 == 0 else ((128 if M > 64 else 64), (128 if Ko > 64 else 64))
    st = torch.empty((-(-M // tile[0]), 2, Ko), device="cuda")
    tb = timeit(lambda: G.conv_fwd(x, w, (s, s), (pad, pad), stat=st, tile=tile))
    st = torch.empty((-(-M // 256), 2, Ko), device="cuda")
    if C % 128 == 0:
        x8 = K.quant_fp8(x, torch.ones(1, device="cuda"))
        w8 = K.quant_fp8(w, torch.ones(1, device="cuda"))
        t8 = timeit(lambda: G.conv_fwd_fp8(x8, w8, (s, s), (pad, pad), stat=st))
        one = torch.ones(1, device="cuda")
        t4 = timeit(lambda: G.conv_fwd4k8(x8, w8, (s, s), (pad, pad), ascale=(one, one)))
    else:
        t8 = t4 = float("nan")
    fl = 2.0 * M * Ko * k * k * C
    print("%2dx%-2d %4d->%-4d k%d: bf16 %7.1f us (%4.0f TF/s)  fp8 8-wave %7.1f us (%4.0f TF/s)  fp8 4-wave %7.1f us "
          "(%4.0f TF/s)" % (H, H, C, Ko, k, tb, fl / tb / 1e6, t8, fl / t8 / 1e6, t4, fl / t4 / 1e6), flush=True)
    del x, w
