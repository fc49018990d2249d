#!/usr/bin/env python3
"""A/B of the streaming pointwise kernel (pw_gemm.hip) against the paths it replaces, on the
ResNet-50 batch-1024 shapes (interleaved rounds in one process, median us):

  fwd    plain 1x1 conv + BN statistics          conv_fwd(stat)            vs pw_conv(stat)
  fwdbn  BN apply (+res) then 1x1 conv + stats   bn_apply + conv_fwd        vs pw_conv(bn_fwd prologue)
  dgrad  bwd-apply then dgrad w/ BN-stat epi     bn_bwd_apply + conv_dgrad  vs pw_conv(bn_bwd prologue)

usage: python tools/pw_bench.py [--batch 1024] [--rounds 5]
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
    from tensorflow_train_distributed_amd.ops import kernels as Kk
    B = args.batch
    # (name, H, K_in, N_out)
    shapes = [("s2 c1 256->64", 56, 256, 64), ("s2 c3 64->256", 56, 64, 256), ("s3 c1 512->128", 28, 512, 128),
              ("s3 c3 128->512", 28, 128, 512), ("s3b1 c1 256->128", 56, 256, 128),
              ("s4 c1 1024->256", 14, 1024, 256), ("s4 c3 256->1024", 14, 256, 1024),
              ("s5 c1 2048->512", 7, 2048, 512)]
    dev = "cuda"

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

    for name, H, Kin, Nout in shapes:
        M = B * H * H
        x = torch.randn(M, Kin, device=dev).bfloat16()
        res = torch.randn(M, Kin, device=dev).bfloat16()
        w = (torch.randn(Nout, Kin, device=dev) / Kin ** 0.5).bfloat16()
        sc = torch.rand(Kin, device=dev) + 0.5
        sh = torch.randn(Kin, device=dev) * 0.1
        h = torch.empty_like(x)
        hm = torch.empty(M * Kin // 8, dtype=torch.uint8, device=dev)
        T128 = -(-M // 128)
        T256 = -(-M // 256)
        part = torch.empty((max(T128, T256), 2, Nout), device=dev)
        x4 = x.view(B, H, H, Kin)
        w4 = w.view(Nout, 1, 1, Kin)
        bm = 256 if G.big_bn(M, Nout, Kin) else 128
        ok = G.pw_rows(Nout, Kin) > 0
        variants = {
            "fwd_old": lambda: G.conv_fwd(x4, w4, stat=part[: -(-M // bm)], tile=(bm, G.big_bn(M, Nout, Kin) or 64)),
            "fwdbn_old": lambda: (Kk.bn_apply(x, sc, sh, residual=res, relu=True, out=h, mask=hm),
                                  G.conv_fwd(h.view(B, H, H, Kin), w4, stat=part[: -(-M // bm)],
                                             tile=(bm, G.big_bn(M, Nout, Kin) or 64))),
        }
        if ok:
            variants["fwd_pw"] = lambda: G.pw_conv(x, w, stat=True)
            variants["fwdbn_pw"] = lambda: G.pw_conv(x, w, prologue=("bn_fwd", sc, sh, res, None, None, h, hm),
                                                     stat=True)
        # backward: this conv's dgrad (dz over Nout channels -> dx over Kin channels)
        g = torch.randn(M, Nout, device=dev).bfloat16()
        yb = torch.randn(M, Nout, device=dev).bfloat16()
        bits = torch.randint(0, 256, (M * Nout // 8,), dtype=torch.uint8, device=dev)
        coef = torch.randn(3, Nout, device=dev) * 0.1
        dz = torch.empty_like(g)
        wt = w.t().contiguous()  # [Kin][Nout]
        y2 = torch.randn(B, H, H, Kin, device=dev).bfloat16()
        bits2 = torch.randint(0, 256, (M * Kin // 8,), dtype=torch.uint8, device=dev)
        dx = torch.randn(B, H, H, Kin, device=dev).bfloat16()
        variants["dgrad_old"] = lambda: (
            _lib.call("ttdk_bn_bwd_apply", g.data_ptr(), None, bits.data_ptr(), yb.data_ptr(), coef.data_ptr(),
                      dz.data_ptr(), M * Nout, Nout, _lib.stream()),
            G.conv_dgrad(dz.view(B, H, H, Nout), wt.view(Kin, 1, 1, Nout), (B, H, H, Kin), out=dx, beta=1,
                         bn_stat=(y2, bits2)))
        if G.pw_rows(Kin, Nout, dma=True) > 0:
            variants["dgrad_pw"] = lambda: G.pw_conv(g, wt, prologue=("bn_bwd", yb, bits, coef, dz), out=dx.view(M, Kin),
                                                     beta=1, bn_stat=(y2, bits2))
        res_t = {k: [] for k in variants}
        for _ in range(args.rounds):
            for k, fn in variants.items():
                fn()
                res_t[k].append(timeit(fn))
        gb = {"fwd": 2 * (M * Kin + M * Nout), "fwdbn": 2 * (3 * M * Kin + M * Nout),
              "dgrad": 2 * (3 * M * Nout + 3 * M * Kin)}
        line = "%-18s M=%-8d" % (name, M)
        for k in variants:
            t = statistics.median(res_t[k])
            line += "  %s %7.1f us (%.2f TB/s)" % (k, t, gb[k.split("_")[0]] / t / 1e6)
        print(line, flush=True)


if __name__ == "__main__":
    main()
