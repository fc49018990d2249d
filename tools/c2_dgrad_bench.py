#!/usr/bin/env python3
"""Standalone ResNet-50 b1024 3x3 (unit-stride) data gradients of the c2 units at stages 3-5:
plain, with the feeding-BN statistics epilogue the engine uses (masked gradient + BN-backward
sums of c1), and (when available) the fp8 e5m2 x e4m3 variant. Prints us / TF/s.
usage: python tools/c2_dgrad_bench.py [--batch 1024]"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
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


def main():
    B = int(sys.argv[sys.argv.index("--batch") + 1]) if "--batch" in sys.argv else 1024
    for name, H, C in (("s3_c2", 28, 128), ("s4_c2", 14, 256), ("s5_c2", 7, 512)):
        dz = (torch.randn(B, H, H, C, device="cuda") * 0.1).bfloat16()
        wt = (torch.randn(C, 3, 3, C, device="cuda") * (9 * C) ** -0.5).bfloat16()
        y1 = torch.randn(B, H, H, C, device="cuda").bfloat16()
        mask = torch.randint(0, 256, (B * H * H * C // 8,), dtype=torch.uint8, device="cuda")
        fl = 2.0 * B * H * H * C * 9 * C
        r = {"shape": name}
        t = timeit(lambda: G.conv_dgrad(dz, wt, (B, H, H, C), (1, 1), (1, 1)))
        r["plain_us"], r["plain_TF"] = round(t, 1), round(fl / t / 1e6)
        t = timeit(lambda: G.conv_dgrad(dz, wt, (B, H, H, C), (1, 1), (1, 1), bn_stat=(y1, mask)))
        r["bnstat_us"], r["bnstat_TF"] = round(t, 1), round(fl / t / 1e6)
        if hasattr(G, "conv_dgrad_fp8"):
            from tensorflow_train_distributed_amd.ops import kernels as K
            one = torch.ones(1, device="cuda")
            dz8 = K.quant_fp8(dz, one, e5m2=True)
            wt8 = K.quant_fp8(wt, one)
            t = timeit(lambda: G.conv_dgrad_fp8(dz8, wt8, (B, H, H, C), (1, 1), (1, 1), bn_stat=(y1, mask)))
            r["fp8_bnstat_us"], r["fp8_bnstat_TF"] = round(t, 1), round(fl / t / 1e6)
            ref = G.conv_dgrad(dz, wt, (B, H, H, C), (1, 1), (1, 1))
            got = G.conv_dgrad_fp8(dz8, wt8, (B, H, H, C), (1, 1), (1, 1))
            r["fp8_rel_err"] = float((got.float() - ref.float()).norm() / ref.float().norm())
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
