#!/usr/bin/env python3
"""Time ResNet-50 (batch 512) conv GEMMs through ops.gemm with forced tile choices and print
us / TF/s / effective GB/s per variant. usage: python tools/conv_bench.py [filter-substring]"""
import sys

import torch

sys.path.insert(0, ".")
from tensorflow_train_distributed_amd.ops import gemm as G  # noqa: E402

B = 512
# name, N, H, W, C, K, R, stride, pad
LAYERS = [
    ("s1_c1_64", B, 56, 56, 256, 64, 1, 1, 0),
    ("s1_c3_64to256", B, 56, 56, 64, 256, 1, 1, 0),
    ("s1_c2_3x3", B, 56, 56, 64, 64, 3, 1, 1),
    ("s2_c3", B, 28, 28, 128, 512, 1, 1, 0),
    ("s2_c1", B, 28, 28, 512, 128, 1, 1, 0),
    ("s3_c3", B, 14, 14, 256, 1024, 1, 1, 0),
    ("s3_c1", B, 14, 14, 1024, 256, 1, 1, 0),
    ("stem", B, 224, 224, 8, 64, 7, 2, 3),
]
TILES = [(0, 0), (256, 256), (256, 128), (128, 128), (128, 64), (64, 128)]


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


def main():
    filt = sys.argv[1] if len(sys.argv) > 1 else ""
    for name, N, H, W, C, K, R, s, p in LAYERS:
        if filt not in name:
            continue
        x = torch.randn(N, H, W, C, device="cuda").bfloat16()
        w = (torch.randn(K, R, R, C, device="cuda") / (R * R * C) ** 0.5).bfloat16()
        y = G.conv_fwd(x, w, (s, s), (p, p))
        P = y.shape[1]
        M = N * P * P
        fl = 2.0 * M * K * R * R * C
        dy = torch.randn_like(y)
        wt = w.permute(3, 1, 2, 0).contiguous()
        byts = {"fwd": 2 * (N * H * W * C + M * K), "dgrad": 2 * (N * H * W * C + M * K),
                "wgrad": 2 * (N * H * W * C + M * K)}
        for op in ("fwd", "dgrad", "wgrad"):
            line = []
            for t in TILES:
                try:
                    if op == "fwd":
                        stat = torch.empty((-(-M // max(64, t[0] or 128)), 2, K), device="cuda")
                        fn = lambda: G.conv_fwd(x, w, (s, s), (p, p), tile=t)  # noqa: E731
                    elif op == "dgrad":
                        fn = lambda: G.conv_dgrad(dy, wt, x.shape, (s, s), (p, p), tile=t)  # noqa: E731
                    else:
                        fn = lambda: G.conv_wgrad(x, dy, w.shape, (s, s), (p, p), tile=t)  # noqa: E731
                    us = timeit(fn)
                    line.append("%s:%6.0fus %4.0fTF %4.1fTB" % ("%dx%d" % t, us, fl / us / 1e6, byts[op] / us / 1e6))
                except Exception as ex:  # noqa: BLE001
                    line.append("%dx%d: n/a" % t)
            print("%-14s %-5s M=%d N=%d K=%d | %s" % (name, op, M, K, R * R * C, " | ".join(line)), flush=True)


if __name__ == "__main__":
    main()
