#!/usr/bin/env python3
"""Time the GEMM kernels on the shapes that matter (random bf16 operands):
4-wave 128x128 kernel (tile=(128,128)) vs the 256x256 LDS-DMA kernel (tile=(256,256)),
plus torch.matmul (hipBLASLt) as a yardstick. Prints TF/s.
usage: gemm_bench.py [--tokens T (BERT rows, default 16384)] [--only SUBSTR]"""
import sys

import torch

sys.path.insert(0, ".")
from tensorflow_train_distributed_amd.ops import gemm as G  # noqa: E402

T = int(sys.argv[sys.argv.index("--tokens") + 1]) if "--tokens" in sys.argv else 16384
ONLY = sys.argv[sys.argv.index("--only") + 1] if "--only" in sys.argv else None
SHAPES = [  # (name, M, N, K, trans_a, trans_b)
    ("sq4096_nt", 4096, 4096, 4096, False, True),
    ("sq8192_nt", 8192, 8192, 8192, False, True),
    ("bert_qkv_fwd", T, 3072, 1024, False, True),
    ("bert_ffn1_fwd", T, 4096, 1024, False, True),
    ("bert_ffn2_fwd", T, 1024, 4096, False, True),
    ("bert_ffn2_dgrad", T, 4096, 1024, False, False),
    ("bert_ffn1_dgrad", T, 1024, 4096, False, False),
    ("bert_ffn1_wgrad", 4096, 1024, T, True, False),
    ("bert_qkv_wgrad", 3072, 1024, T, True, False),
    # ResNet-50 batch-256 1x1 conv GEMMs (fwd: pixels x Cout x Cin)
    ("r50_s2_c3_fwd", 802816, 256, 64, False, True),
    ("r50_s2_c1_fwd", 802816, 64, 256, False, True),
    ("r50_s3_c3_fwd", 200704, 512, 128, False, True),
    ("r50_s3_c1_fwd", 200704, 128, 512, False, True),
    ("r50_s4_c3_fwd", 50176, 1024, 256, False, True),
    ("r50_s4_c1_fwd", 50176, 256, 1024, False, True),
    ("r50_s5_c3_fwd", 12544, 2048, 512, False, True),
    ("r50_s4_c3_wgrad", 1024, 256, 50176, True, False),
    ("r50_s3_c3_wgrad", 512, 128, 200704, True, False),
]


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main():
    for name, M, N, K, ta, tb in SHAPES:
        if ONLY and ONLY not in name:
            continue
        a = (torch.rand((K, M) if ta else (M, K), device="cuda") * 2 - 1).bfloat16()
        b = (torch.rand((N, K) if tb else (K, N), device="cuda") * 2 - 1).bfloat16()
        fl = 2.0 * M * N * K
        res = []
        wgrad = ta
        for tile in ((128, 128), (256, 256)):
            if tile[0] == 256 and (M < 256 or N < 256):
                res.append("256 n/a")
                continue
            if wgrad:
                out = torch.empty(M, N, device="cuda")
                sp = G.gemm_wgrad_splits(M, N, K) if tile[0] == 128 else max(1, 256 // ((M // 256) * (N // 256)))
                f = lambda: G.gemm(a, b, trans_a=ta, trans_b=tb, out=out, splits=sp, tile=tile)  # noqa: E731
            else:
                out = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
                f = lambda: G.gemm(a, b, trans_a=ta, trans_b=tb, out=out, tile=tile)  # noqa: E731
            ms = timeit(f)
            res.append("%s %.3f ms %.0f TF/s" % (tile[0], ms, fl / ms / 1e9))
            if tile[0] == 256 and not wgrad:  # one-tile-per-workgroup kernel (persistent path off)
                from tensorflow_train_distributed_amd.ops import _lib
                prev = _lib.query("ttdk_set_big_pers", 0)
                ms = timeit(f)
                _lib.query("ttdk_set_big_pers", prev)
                res.append("256np %.3f ms %.0f TF/s" % (ms, fl / ms / 1e9))
                prev = _lib.query("ttdk_set_big_pers", 2)
                ms = timeit(f)
                _lib.query("ttdk_set_big_pers", prev)
                res.append("256p-noovl %.3f ms %.0f TF/s" % (ms, fl / ms / 1e9))
        at = a.t() if ta else a
        bt = b.t() if tb else b
        ms = timeit(lambda: torch.matmul(at, bt))
        res.append("torch %.3f ms %.0f TF/s" % (ms, fl / ms / 1e9))
        if not ta and tb and K % 128 == 0:  # fp8 e4m3 on the block-scaled MFMA (same NT layout)
            from tensorflow_train_distributed_amd.ops import kernels as KK
            one = torch.ones(1, device="cuda")
            a8, b8 = KK.quant_fp8(a, one), KK.quant_fp8(b, one)
            o8 = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
            ms = timeit(lambda: G.gemm_fp8(a8, b8, out=o8))
            res.append("fp8 %.3f ms %.0f TF/s" % (ms, fl / ms / 1e9))
        # correctness spot check of the 256 path
        out = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
        G.gemm(a, b, trans_a=ta, trans_b=tb, out=out, tile=(256, 256) if min(M, N) >= 256 else (128, 128))
        ref = torch.matmul(at, bt)
        err = float((out.float() - ref.float()).abs().max())
        print("%-16s M=%5d N=%5d K=%5d | %s | maxerr %.3g" % (name, M, N, K, " | ".join(res), err), flush=True)


if __name__ == "__main__":
    main()
