#!/usr/bin/env python3
"""Cost of the fused epilogue pieces of the ResNet c1 data gradients (1x1, stride 1) at
b1024: plain store, + accumulate (beta), + BN-backward statistics of the feeding unit (y, mask),
+ the projection BN's second statistics (y2). usage: dgrad_epi_probe.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from tensorflow_train_distributed_amd.ops import gemm as G  # noqa: E402


def timeit(fn, n=5):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n * 1e3


def main():
    dev = "cuda"
    for (B, H, C, K) in ((1024, 28, 512, 128), (1024, 14, 1024, 256), (1024, 7, 2048, 512)):
        dz = torch.randn(B, H, H, K, device=dev).bfloat16()
        wt = (torch.randn(C, 1, 1, K, device=dev) * 0.05).bfloat16()
        out = torch.randn(B, H, H, C, device=dev).bfloat16()
        fy = torch.randn(B, H, H, C, device=dev).bfloat16()
        fy2 = torch.randn(B, H, H, C, device=dev).bfloat16()
        fm = torch.randint(0, 256, (B * H * H * C // 8,), dtype=torch.uint8, device=dev)
        xs = (B, H, H, C)
        v = {
            "plain": lambda: G.conv_dgrad(dz, wt, xs, out=out),
            "beta": lambda: G.conv_dgrad(dz, wt, xs, out=out, beta=1),
            "beta+stat": lambda: G.conv_dgrad(dz, wt, xs, out=out, beta=1, bn_stat=(fy, fm)),
            "beta+stat+stat2": lambda: G.conv_dgrad(dz, wt, xs, out=out, beta=1, bn_stat=(fy, fm), bn_stat2=fy2),
        }
        M = B * H * H
        wt2 = wt.view(C, K)
        if G.pw_rows(C, K, dma=True):  # streaming kernel, LDS-DMA epilogue (no second statistics source)
            v["pw beta+stat"] = lambda: G.pw_conv(dz.view(M, K), wt2, out=out.view(M, C), beta=1, bn_stat=(fy, fm))
        res = []
        for k, f in v.items():
            t = timeit(f)
            nb = M * K * 2 + M * C * 2 * (1 + (k != "plain") + (k.count("stat") > 0) + (k.count("stat2") > 0)) \
                + (M * C // 8 if "stat" in k else 0)
            res.append("%s %.1f us (%.2f TB/s)" % (k, t, nb / t / 1e6))
        print("M=%d N=%d K=%d | %s" % (M, C, K, " | ".join(res)), flush=True)


if __name__ == "__main__":
    main()
