#!/usr/bin/env python3
"""ResNet-50 b1024 forward 1x1 convs (stage 4 / 5, unit stride) as GEMMs: the 8-wave 256-row conv
kernel with its BN-statistics epilogue (ops.gemm.conv_fwd, as the engine calls it) vs the 4-wave
AGPR GEMM (ops.gemm.gemm4w, plain store) on the same operands. HIP events, median of 10."""
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
for hw, cin, cout in ((14, 256, 1024), (14, 1024, 256), (7, 512, 2048), (7, 2048, 512), (14, 1024, 512)):
    M = B * hw * hw
    x = (torch.randn(B, hw, hw, cin, device="cuda") * 0.5).bfloat16()
    w = (torch.randn(cout, 1, 1, cin, device="cuda") * 0.05).bfloat16()
    big = G.big_bn(M, cout, cin)
    T = -(-M // 256)
    part = torch.empty((T, 2, cout), dtype=torch.float32, device="cuda")
    y = torch.empty((B, hw, hw, cout), dtype=torch.bfloat16, device="cuda")
    f_conv = lambda: G.conv_fwd(x, w, stat=part, tile=(256, big), out=y)  # noqa: E731
    x2, w2, y2 = x.view(M, cin), w.view(cout, cin), y.view(M, cout)
    f_g4 = lambda: G.gemm4w(x2, w2, out=y2)  # noqa: E731
    tc, tg = t(f_conv), t(f_g4)
    fl = 2.0 * M * cin * cout
    print("M=%7d N=%5d K=%5d  conv_fwd(stat) %7.1f us %5.0f TF/s   gemm4w %7.1f us %5.0f TF/s  (%.2fx)"
          % (M, cout, cin, tc, fl / tc / 1e6, tg, fl / tg / 1e6, tc / tg))
