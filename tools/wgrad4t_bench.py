#!/usr/bin/env python3
"""ResNet-50 b1024 convolution weight gradients: the 4-wave transposed-read kernel with the im2col
gather (ops.gemm.conv_wgrad4t, split-K summed in the launch) vs the previous path (8-wave 256-row /
128-tile kernels + split-K fold launches, TTD_WGRAD4T=0 policy), standalone, HIP events.
usage: wgrad4t_bench.py [--batch B] [--wgs W1,W2,..] [--rounds R]"""
import sys

import torch

sys.path.insert(0, ".")
from tensorflow_train_distributed_amd.ops import gemm as G  # noqa: E402


def arg(name, default):
    return sys.argv[sys.argv.index(name) + 1] if name in sys.argv else default


B = int(arg("--batch", "1024"))
WGS = [int(v) for v in arg("--wgs", "128").split(",")]
ROUNDS = int(arg("--rounds", "2"))
# (name, H, C, K, R, stride): conv input H x H x C, K filters of R x R
SHAPES = [("s5_c2", 7, 512, 512, 3, 1), ("s5b1_c2", 14, 512, 512, 3, 2), ("s5_c1", 7, 2048, 512, 1, 1),
          ("s5_c3", 7, 512, 2048, 1, 1), ("s5_cd", 14, 1024, 2048, 1, 2), ("s5b1_c1", 14, 1024, 512, 1, 1),
          ("s4_c2", 14, 256, 256, 3, 1), ("s4b1_c2", 28, 256, 256, 3, 2), ("s4_c1", 14, 1024, 256, 1, 1),
          ("s4_c3", 14, 256, 1024, 1, 1), ("s4_cd", 28, 512, 1024, 1, 2), ("s4b1_c1", 28, 512, 256, 1, 1),
          ("s3_c3", 28, 128, 512, 1, 1), ("s3_cd", 56, 256, 512, 1, 2),
          # fewer than 256 output channels: the 128-row tile form
          ("s3_c2", 28, 128, 128, 3, 1), ("s3b1_c2", 56, 128, 128, 3, 2), ("s3_c1", 28, 512, 128, 1, 1),
          ("s3b1_c1", 56, 256, 128, 1, 1), ("s2_c2", 56, 64, 64, 3, 1), ("s2_c1", 56, 256, 64, 1, 1)]
ONLY = arg("--only", "")


def timeit(fn, iters=10):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1000.0


def main():
    tot = {}
    for name, H, C, K, R, st in SHAPES:
        if ONLY and not any(o in name for o in ONLY.split(",")):
            continue
        pad = R // 2
        P = (H + 2 * pad - R) // st + 1
        x = (torch.rand((B, H, H, C), device="cuda") * 2 - 1).bfloat16()
        dy = (torch.rand((B, P, P, K), device="cuda") * 2 - 1).bfloat16()
        w = (K, R, R, C)
        out = torch.empty(w, device="cuda")
        g = G.conv_geom(x.shape, w, (st, st), (pad, pad))
        arms = {}
        cus = {"old": 256}  # (the previous kernels launch >= 256 workgroups on these shapes)
        old = G._WGRAD4T
        G._WGRAD4T = 0
        arms["old"] = lambda: G.conv_wgrad(x, dy, w, (st, st), (pad, pad), out=out)
        if G.conv_wgrad4t_ok(g, mode=2):
            for wg in WGS:
                sp = G.conv_wgrad4t_splits(g, target_blocks=wg)
                arms["g4t@%d(s%d)" % (wg, sp)] = (lambda sp=sp: G.conv_wgrad4t(x, dy, w, (st, st), (pad, pad),
                                                                               out=out, splits=sp))
                # CU-time of the launch (what it costs the data-gradient chain next to it)
                bm = G.wgrad4t_rows(K)
                cus[("g4t@%d(s%d)" % (wg, sp))] = min(256, -(-K // bm) * -(-(R * R * C) // 256) * sp)
        res = {k: [] for k in arms}
        for _ in range(ROUNDS):
            for k, f in arms.items():
                res[k].append(timeit(f))
        G._WGRAD4T = old
        fl = 2.0 * K * R * R * C * B * P * P
        line = "%-8s M=%4d N=%4d K=%7d" % (name, K, R * R * C, B * P * P)
        for k, v in res.items():
            t = min(v)
            tot[k.split("@")[0]] = tot.get(k.split("@")[0], 0.0) + (t if "@" not in k or k.endswith(
                "(s%d)" % G.conv_wgrad4t_splits(g, target_blocks=WGS[0])) else 0.0)
            line += "  %s %7.1f us %5.0f TF/s %5.1f CU-ms" % (k, t, fl / t / 1e6, t * cus.get(k, 256) / 1e3)
        print(line, flush=True)
        del x, dy, out
    print("totals (first wgs):", {k: round(v, 1) for k, v in tot.items()})


if __name__ == "__main__":
    main()
