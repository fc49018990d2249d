#!/usr/bin/env python3
"""fp8 weight gradients at the ResNet-50 b1024 shapes of precision="fp8": the 4-wave transposed-read
kernel's fp8 form (gemm4t.hip gemm4t8_kernel) vs the 8-wave 256x128 kernel (conv_wgrad.hip), and
the bf16 4-wave kernel on the same shape for reference. HIP events, mean of 10 launches, at the
engine's split choice and at a 256-workgroup target (standalone: the whole chip).
usage: python tools/wgrad_fp8_bench.py [batch]"""
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


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    dev = torch.device("cuda", 0)
    # (name, H, C, K, R, stride): input H x H x C, K output channels
    shapes = [("s2_c2 3x3", 28, 128, 128, 3, 1), ("s3_c2 3x3", 14, 256, 256, 3, 1), ("s4_c2 3x3", 7, 512, 512, 3, 1),
              ("s3_c2 3x3/2", 28, 256, 256, 3, 2), ("s4_c2 3x3/2", 14, 512, 512, 3, 2),
              ("s3_c1 1x1", 14, 1024, 256, 1, 1), ("s3_c3 1x1", 14, 256, 1024, 1, 1),
              ("s4_c1 1x1", 7, 2048, 512, 1, 1), ("s4_c3 1x1", 7, 512, 2048, 1, 1), ("s2_c1 1x1", 28, 512, 128, 1, 1)]
    one = torch.ones(1, device=dev)
    print("%-14s %9s %9s %9s %9s   %s" % ("shape", "4w-fp8", "8w-fp8", "4w-bf16", "fp8 x", "TF/s 4w-fp8"))
    for name, H, C, Kc, R, s in shapes:
        pad = 1 if R == 3 else 0
        x = torch.randn(B, H, H, C, device=dev).relu().bfloat16()
        P = (H + 2 * pad - R) // s + 1
        dy = (torch.randn(B, P, P, Kc, device=dev) * 1e-3).bfloat16()
        x8 = K.quant_fp8(x, one * 64)
        dy8 = K.quant_fp8(dy, one * 2 ** 20, e5m2=True)
        ws = (Kc, R, R, C)
        inv = (one, one)
        G._WGRAD4T8 = True
        t4 = timeit(lambda: G.conv_wgrad_fp8(x8, dy8, ws, (s, s), (pad, pad), ascale=inv))
        G._WGRAD4T8 = False
        t8 = timeit(lambda: G.conv_wgrad_fp8(x8, dy8, ws, (s, s), (pad, pad), ascale=inv))
        G._WGRAD4T8 = True
        tb = timeit(lambda: G.conv_wgrad(x, dy, ws, (s, s), (pad, pad)))
        flop = 2.0 * Kc * R * R * C * B * P * P
        print("%-14s %9.1f %9.1f %9.1f %9.2f   %.0f" % (name, t4, t8, tb, t8 / t4, flop / t4 / 1e6), flush=True)
        del x, dy, x8, dy8
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
