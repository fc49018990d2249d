#!/usr/bin/env python3
"""A/B of the halo 3x3 kernel (conv3_halo.hip) against the paths it replaces on the ResNet-50
stage-2 shape (56x56, 64 -> 64, batch B; interleaved rounds in one process, median us):

  fwd     plain conv + BN statistics                 conv_fwd(stat)                vs conv3_halo(stat)
  fwdbn   BN apply + ReLU, then conv + statistics    bn_apply + conv_fwd(stat)     vs conv3_halo(bn_fwd)
  dgrad   BN bwd-apply, then dgrad w/ BN-stat epi    bn_bwd_apply + conv_dgrad     vs conv3_halo(flip, bn_bwd)

usage: python tools/conv3_bench.py [--batch 1024] [--rounds 5]
"""
import argparse
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--rounds", type=int, default=5)
    args = ap.parse_args()
    from tensorflow_train_distributed_amd.ops import _lib
    from tensorflow_train_distributed_amd.ops import gemm as G
    from tensorflow_train_distributed_amd.ops import kernels as K
    B, H, W, C, N = args.batch, 56, 56, 64, 64
    M = B * H * W
    dev = "cuda"
    x = torch.randn(B, H, W, C, device=dev).bfloat16()
    w = (torch.randn(N, 3, 3, C, device=dev) / (9 * C) ** 0.5).bfloat16()
    wt = K.krsc_to_crsk(w)
    sc = torch.rand(C, device=dev) + 0.5
    sh = torch.randn(C, device=dev) * 0.1
    h = torch.empty_like(x)
    hm = torch.empty(M * C // 8, dtype=torch.uint8, device=dev)
    bm = 128
    part = torch.empty((-(-M // bm), 2, N), device=dev)
    g = torch.randn(B, H, W, N, device=dev).bfloat16()
    y = torch.randn(B, H, W, N, device=dev).bfloat16()
    coef = torch.randn(3, N, device=dev) * 0.1
    dz = torch.empty_like(g)
    fy = torch.randn(B, H, W, C, device=dev).bfloat16()
    fm = torch.randint(0, 256, (M * C // 8,), dtype=torch.uint8, device=dev)

    def ev():
        return torch.cuda.Event(enable_timing=True)

    def timeit(fn, n=3):
        s, e = ev(), ev()
        s.record()
        for _ in range(n):
            fn()
        e.record()
        torch.cuda.synchronize()
        return s.elapsed_time(e) / n * 1e3

    variants = {
        "fwd_old": lambda: G.conv_fwd(x, w, (1, 1), (1, 1), stat=part, tile=(bm, 64)),
        "fwd_c3": lambda: G.conv3_halo(x, w, stat=True),
        "fwdbn_old": lambda: (K.bn_apply(x.view(M, C), sc, sh, relu=True, out=h.view(M, C), mask=hm),
                              G.conv_fwd(h, w, (1, 1), (1, 1), stat=part, tile=(bm, 64))),
        "fwdbn_c3": lambda: G.conv3_halo(x, w, prologue=("bn_fwd", sc, sh, h, hm), stat=True),
        "dgrad_old": lambda: (_lib.call("ttdk_bn_bwd_apply", g.data_ptr(), None, None, y.data_ptr(), coef.data_ptr(),
                                        dz.data_ptr(), M * N, N, _lib.stream()),
                              G.conv_dgrad(dz, wt, (B, H, W, C), (1, 1), (1, 1), bn_stat=(fy, fm))),
        "dgrad_c3": lambda: G.conv3_halo(g, wt, flip=True, prologue=("bn_bwd", y, None, coef, dz), bn_stat=(fy, fm)),
        "dgrad_c3p0": lambda: (_lib.call("ttdk_bn_bwd_apply", g.data_ptr(), None, None, y.data_ptr(), coef.data_ptr(),
                                         dz.data_ptr(), M * N, N, _lib.stream()),
                               G.conv3_halo(dz, wt, flip=True, bn_stat=(fy, fm))),
        "dg_gemm": lambda: G.conv_dgrad(dz, wt, (B, H, W, C), (1, 1), (1, 1), bn_stat=(fy, fm)),
        "dg_c3": lambda: G.conv3_halo(dz, wt, flip=True, bn_stat=(fy, fm)),
    }
    res = {k: [] for k in variants}
    for _ in range(args.rounds):
        for k, fn in variants.items():
            fn()
            res[k].append(timeit(fn))
    flop = 2.0 * M * N * 9 * C
    for k in variants:
        t = statistics.median(res[k])
        print("%-10s %8.1f us  %6.0f TF/s" % (k, t, flop / t / 1e6), flush=True)


if __name__ == "__main__":
    main()
