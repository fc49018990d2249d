#!/usr/bin/env python3
"""Cost of the BN-statistics epilogue on the ResNet-50 b1024 forward 1x1-conv GEMMs: the
256-row kernel with stat rows (as the engine runs them) vs the same GEMM with a plain store
(one-tile kernel and the persistent kernel) vs hipBLASLt (torch.matmul).
usage: python tools/epi_cost_bench.py"""
import sys

import torch

sys.path.insert(0, ".")
from tensorflow_train_distributed_amd.ops import gemm as G  # noqa: E402

SHAPES = [(200704, 256, 1024), (50176, 2048, 512), (200704, 1024, 256), (50176, 512, 2048), (802816, 256, 512),
          (802816, 128, 512), (200704, 512, 1024)]


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
    from tensorflow_train_distributed_amd import _native
    hip = _native.hip()
    for M, N, K in SHAPES:
        x = (torch.rand(M, K, device="cuda") * 2 - 1).bfloat16()
        w = (torch.rand(N, K, device="cuda") * 2 - 1).bfloat16()
        bn = G.big_bn(M, N, K)
        out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        st = torch.empty((-(-M // 256), 2, N), device="cuda")
        fl = 2.0 * M * N * K
        r = {}
        r["stat"] = timeit(lambda: G.gemm(x, w, trans_b=True, out=out, stat=st, tile=(256, bn)))
        hip.ttdk_set_big_pers(0)
        r["plain"] = timeit(lambda: G.gemm(x, w, trans_b=True, out=out, tile=(256, bn)))
        hip.ttdk_set_big_pers(1)
        r["plain_pers"] = timeit(lambda: G.gemm(x, w, trans_b=True, out=out, tile=(256, bn)))
        r["torch"] = timeit(lambda: torch.matmul(x, w.t(), out=out))
        floor = (2 * (M * K + N * K + M * N)) / 5.5e6
        print("M=%-7d N=%-5d K=%-5d BN=%d  " % (M, N, K, bn) +
              "  ".join("%s %6.1f us (%4.0f TF/s)" % (k, v, fl / v / 1e6) for k, v in r.items()) +
              "  | HBM floor %.1f us" % floor, flush=True)
        del x, w, out, st


if __name__ == "__main__":
    main()
