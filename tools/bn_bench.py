#!/usr/bin/env python3
"""Standalone HBM rate of the BatchNorm streaming passes (batchnorm.hip apply_kernel /
bwd_apply_kernel) at the ResNet-50 b1024 activation shapes, next to a plain device copy of the
same bytes. HIP events, median of 20 launches.

    python tools/bn_bench.py [--batch 1024]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from tensorflow_train_distributed_amd.ops import kernels as K  # noqa: E402


def timeit(fn, n=20, pre=None):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(n):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        if pre is not None:
            pre()  # a producer that has just written the pass's input (as in the training step)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    ts.sort()
    return ts[len(ts) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--after-write", action="store_true",
                    help="re-write the input right before every timed pass (a producer kernel in front)")
    ap.add_argument("--shapes", default="", help="comma list of HWxC, e.g. 28x128,56x64")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    N = a.batch
    shapes = [(56, 256), (56, 64), (28, 512), (28, 128), (14, 1024), (14, 256), (7, 2048), (7, 512)]
    if a.shapes:
        shapes = [tuple(int(v) for v in s_.split("x")) for s_ in a.shapes.split(",")]
    print("%-14s %-28s %9s %8s %8s" % ("shape", "pass", "us", "GB", "TB/s"))
    for hw, C in shapes:
        M = N * hw * hw
        y = torch.randn(M, C, device=dev).bfloat16()
        r = torch.randn(M, C, device=dev).bfloat16()
        g = torch.randn(M, C, device=dev).bfloat16()
        sc = torch.rand(C, device=dev) + 0.5
        sh = torch.randn(C, device=dev)
        coef = torch.randn(3, C, device=dev)
        out = torch.empty_like(y)
        dz = torch.empty_like(y)
        mask = torch.empty(M * C // 8, dtype=torch.uint8, device=dev)
        e = M * C
        src = torch.randn(M, C, device=dev).bfloat16() if a.after_write else None
        pre = (lambda: y.copy_(src)) if a.after_write else None
        cases = [
            ("copy", lambda: out.copy_(y), 4 * e),
            ("apply relu+mask", lambda: K.bn_apply(y, sc, sh, relu=True, out=out, mask=mask), 4 * e + e // 8),
            ("apply res relu+mask", lambda: K.bn_apply(y, sc, sh, residual=r, relu=True, out=out, mask=mask),
             6 * e + e // 8),
            ("bwd_apply (g, y -> dz)", lambda: K._lib.call("ttdk_bn_bwd_apply_q8", g.data_ptr(), None, None,
                                                            y.data_ptr(), coef.data_ptr(), dz.data_ptr(), None, None,
                                                            e, C, K._s()), 6 * e),
            ("bwd_apply mask", lambda: K._lib.call("ttdk_bn_bwd_apply", g.data_ptr(), None, mask.data_ptr(),
                                                    y.data_ptr(), coef.data_ptr(), dz.data_ptr(), e, C, K._s()),
             6 * e + e // 8),
        ]
        for name, fn, nbytes in cases:
            us = timeit(fn, pre=pre)
            print("%-14s %-28s %9.1f %8.3f %8.2f" % ("%dx%d" % (M, C), name, us, nbytes / 1e9, nbytes / us / 1e6))
        del y, r, g, out, dz, mask, src
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
