#!/usr/bin/env python3
"""ResNet-50 b1024 forward convs that run on the 256-row kernel (ops.gemm.conv_fwd with its BN
statistics epilogue, as the engine called them before round 6) vs the 4-wave GEMM with the im2col
gather and BN-statistics register epilogue (ops.gemm.conv_fwd4w). HIP events, median of 10."""
import sys

import torch

sys.path.insert(0, ".")
from tensorflow_train_distributed_amd.ops import gemm as G  # noqa: E402


def t(fn, n=10):
    fn()
    torch.cuda.synchronize()
    r = []
    for _ in range(n):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        r.append(a.elapsed_time(b) * 1e3)
    return sorted(r)[n // 2]


B = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
# (name, H, C, K, R, stride)
SHAPES = [("s3b1_c2", 56, 128, 128, 3, 2), ("s3_cd", 56, 256, 512, 1, 2), ("s4b1_c2", 28, 256, 256, 3, 2),
          ("s4_c2", 14, 256, 256, 3, 1), ("s4_cd", 28, 512, 1024, 1, 2), ("s4_c1", 14, 1024, 256, 1, 1),
          ("s4_c3", 14, 256, 1024, 1, 1), ("s5b1_c2", 14, 512, 512, 3, 2), ("s5_c2", 7, 512, 512, 3, 1),
          ("s5_cd", 14, 1024, 2048, 1, 2), ("s5_c1", 7, 2048, 512, 1, 1), ("s5_c3", 7, 512, 2048, 1, 1)]
tot = [0.0, 0.0]
for name, H, C, K, R, st in SHAPES:
    pad = R // 2
    x = (torch.randn(B, H, H, C, device="cuda") * 0.5).bfloat16()
    w = (torch.randn(K, R, R, C, device="cuda") * 0.05).bfloat16()
    g = G.conv_geom(x.shape, w.shape, (st, st), (pad, pad))
    M = g.N * g.P * g.Q
    big = G.big_bn(M, K, R * R * C)
    part = torch.empty((-(-M // 256), 2, K), dtype=torch.float32, device="cuda")
    y = torch.empty((g.N, g.P, g.Q, K), dtype=torch.bfloat16, device="cuda")
    f_old = lambda: G.conv_fwd(x, w, (st, st), (pad, pad), stat=part, tile=(256, big), out=y)  # noqa: E731
    f_new = lambda: G.conv_fwd4w(x, w, (st, st), (pad, pad), out=y)  # noqa: E731
    to, tn = t(f_old), t(f_new)
    tot[0] += to
    tot[1] += tn
    fl = 2.0 * M * K * R * R * C
    print("%-8s M=%7d N=%5d K=%5d  conv_fwd %7.1f us %5.0f TF/s  conv_fwd4w %7.1f us %5.0f TF/s  (%.2fx)"
          % (name, M, K, R * R * C, to, fl / to / 1e6, tn, fl / tn / 1e6, to / tn), flush=True)
print("total conv_fwd %.1f us, conv_fwd4w %.1f us" % tuple(tot))

# unit-stride 3x3 data gradients with the feeding-BN epilogue (conv_dgrad(bn_stat=...)): the
# 256-row gather kernel vs the 4-wave kernel (TTD_DGRAD4W policy forced per arm)
print()
tot = [0.0, 0.0]
for name, H, C, K in (("s4_c2", 14, 256, 256), ("s5_c2", 7, 512, 512)):
    dy = (torch.randn(B, H, H, K, device="cuda") * 0.5).bfloat16()
    wt = (torch.randn(C, 3, 3, K, device="cuda") * 0.05).bfloat16()
    y = (torch.randn(B, H, H, C, device="cuda")).bfloat16()
    mask = torch.randint(0, 256, (B * H * H * C // 8,), dtype=torch.uint8, device="cuda")
    out = torch.empty((B, H, H, C), dtype=torch.bfloat16, device="cuda")
    res = []
    for mode in (0, 2):
        G._DGRAD4W = mode
        res.append(t(lambda: G.conv_dgrad(dy, wt, (B, H, H, C), (1, 1), (1, 1), out=out, bn_stat=(y, mask))))
    G._DGRAD4W = 1
    fl = 2.0 * B * H * H * C * 9 * K
    tot[0] += res[0]
    tot[1] += res[1]
    print("%-8s dgrad M=%7d N=%5d K=%5d  256-row %7.1f us %5.0f TF/s  4-wave %7.1f us %5.0f TF/s  (%.2fx)"
          % (name, B * H * H, C, 9 * K, res[0], fl / res[0] / 1e6, res[1], fl / res[1] / 1e6, res[0] / res[1]), flush=True)
print("total 256-row %.1f us, 4-wave %.1f us" % tuple(tot))
