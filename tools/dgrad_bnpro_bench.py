#!/usr/bin/env python3
"""A/B of the BN-backward operand prologue on the 256-row dgrad at ResNet-50 b1024 shapes:
(a) bwd_apply pass (dz = a*g + b*y + c stored) + plain dgrad, vs (b) one dgrad that forms dz
in LDS and stores it. Times per launch pair (HIP events) and the HBM bytes the pair must move.
usage: python tools/dgrad_bnpro_bench.py [--only=s3_c1,s4_c3]"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


_ONLY = [a.split("=", 1)[1] for a in sys.argv[1:] if a.startswith("--only=")]
_ONLY = _ONLY[0].split(",") if _ONLY else []


def timed(fn, iters=10):
    for _ in range(2):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


def main():
    from tensorflow_train_distributed_amd.ops import _lib
    from tensorflow_train_distributed_amd.ops import gemm as G
    dev = torch.device("cuda", 0)
    B = 1024
    res = []
    # (name, H, K = dz channels, C = dx channels, feed epilogue)
    for name, H, K, C, feed in [("s3_c3", 28, 512, 128, False), ("s4_c3", 14, 1024, 256, False),
                                ("s5_c3", 7, 2048, 512, False), ("s3_c1", 28, 128, 512, True),
                                ("s4_c1", 14, 256, 1024, True), ("s5_c1", 7, 512, 2048, True),
                                ("s3b1_c1", 56, 128, 256, True)]:
        if _ONLY and name not in _ONLY:
            continue
        g = torch.randn(B, H, H, K, device=dev).bfloat16()
        y = torch.randn(B, H, H, K, device=dev).bfloat16()
        coef = torch.randn(3, K, device=dev) * 0.1
        w = (torch.randn(K, 1, 1, C, device=dev) / K ** 0.5).bfloat16()
        wt = w.permute(3, 1, 2, 0).contiguous()
        dz = torch.empty_like(g)
        out = torch.empty(B, H, H, C, device=dev).bfloat16()
        kw = {}
        if feed:
            fy = torch.randn(B, H, H, C, device=dev).bfloat16()
            mask = torch.randint(0, 255, (B * H * H * C // 8,), device=dev, dtype=torch.uint8)
            kw = dict(out=out, beta=1, bn_stat=(fy, mask))
        M = B * H * H

        def unfused():
            _lib.call("ttdk_bn_bwd_apply", g.data_ptr(), None, None, y.data_ptr(), coef.data_ptr(), dz.data_ptr(),
                      M * K, K, _lib.stream())
            G.conv_dgrad(dz, wt, (B, H, H, C), **kw)

        def fused():
            G.conv_dgrad(g, wt, (B, H, H, C), bn_pro=(y, coef, dz), **kw)
        ta, tb = timed(unfused), timed(fused)
        X, Y = M * K * 2, M * C * 2
        by_a = 3 * X + X + (3 * Y + Y // 16 if feed else Y)  # pass: g, y in, dz out; dgrad: dz in (+ epilogue)
        by_b = 3 * X + (3 * Y + Y // 16 if feed else Y)
        res.append({"shape": name, "unfused_us": round(ta, 1), "fused_us": round(tb, 1),
                    "speedup": round(ta / tb, 3), "unfused_TBps": round(by_a / ta / 1e6, 2),
                    "fused_TBps": round(by_b / tb / 1e6, 2)})
        print(json.dumps(res[-1]), flush=True)


if __name__ == "__main__" and "--fwd" not in sys.argv:
    main()


def forward_ab():
    """Forward: BN apply pass (+ residual + ReLU + mask) then the next 1x1 conv with BN statistics,
    vs conv_fwd_bnpro (the apply formed in the conv's operand tile)."""
    from tensorflow_train_distributed_amd.ops import gemm as G
    from tensorflow_train_distributed_amd.ops import kernels as K
    dev = torch.device("cuda", 0)
    B = 1024
    for name, H, C, Kout, proj in [("s3_c3->c1", 28, 512, 128, False), ("s3->s4b1_c1", 28, 512, 256, False),
                                   ("s4_c3->c1", 14, 1024, 256, False), ("s4b1_proj", 14, 1024, 256, True)]:
        M = B * H * H
        y3 = torch.randn(B, H, H, C, device=dev).bfloat16()
        r = torch.randn(B, H, H, C, device=dev).bfloat16()
        sc, sh = torch.rand(C, device=dev) + 0.5, torch.randn(C, device=dev) * 0.1
        coef = torch.cat([sc, sh, sc, sh]) if proj else torch.cat([sc, sh])
        w = (torch.randn(Kout, 1, 1, C, device=dev) / C ** 0.5).bfloat16()
        h = torch.empty_like(y3)
        hm = torch.empty(M * C // 8, dtype=torch.uint8, device=dev)
        T = -(-M // 256)
        partial = torch.empty((T, 2, Kout), device=dev)

        def unfused():
            K.bn_apply(y3.view(M, C), sc, sh, residual=r.view(M, C), residual_bn=(sc, sh) if proj else None,
                       relu=True, out=h.view(M, C), mask=hm)
            G.conv_fwd(h, w, stat=partial, tile=(256, G.big_bn(M, Kout, C)))

        def fused():
            G.conv_fwd_bnpro(y3, w, coef, r, h, hm, proj=proj)
        ta, tb = timed(unfused), timed(fused)
        print(json.dumps({"shape": name, "unfused_us": round(ta, 1), "fused_us": round(tb, 1),
                          "speedup": round(ta / tb, 3)}), flush=True)


if __name__ == "__main__" and "--fwd" in sys.argv:
    forward_ab()
