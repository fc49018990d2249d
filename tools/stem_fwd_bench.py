#!/usr/bin/env python3
"""Stem forward at batch N: dedicated kernel (stem_fwd.hip) vs the generic implicit-GEMM conv
with the BN-statistics epilogue. usage: stem_fwd_bench.py [N]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def bench_fwd(N=1024):
    import torch
    from tensorflow_train_distributed_amd.ops import gemm as G
    x = torch.zeros(N, 224, 224, 8, device="cuda", dtype=torch.bfloat16)
    x[..., :3] = torch.randn(N, 224, 224, 3, device="cuda").bfloat16()
    w = (torch.randn(64, 7, 7, 8, device="cuda") * 0.1).bfloat16()
    w[..., 3:] = 0
    bm = 256 if G.big_bn(N * 112 * 112, 64, 392) else 128
    T = -(-N * 112 * 112 // bm)
    stat = torch.empty((T, 2, 64), device="cuda")
    out = {}
    for name, f in (("generic", lambda: G.conv_fwd(x, w, (2, 2), (3, 3), stat=stat, tile=(bm, G.big_bn(N * 112 * 112, 64, 392) or 64))),
                    ("stem_fwd", lambda: G.stem_fwd(x, w))):
        for _ in range(3):
            f()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(10):
            f()
        e.record()
        torch.cuda.synchronize()
        out[name] = s.elapsed_time(e) / 10 * 1e3
    print("stem fwd b%d: generic %.1f us, stem_fwd %.1f us" % (N, out["generic"], out["stem_fwd"]), flush=True)


if __name__ == "__main__":
    bench_fwd(int(sys.argv[1]) if len(sys.argv) > 1 else 1024)
