#!/usr/bin/env python3
"""Time BERT-Large weight-gradient GEMMs (dW = dy^T . x, fp32 out, + bias column sums) on the
engine's entry (ops.gemm.gemm_wgrad_bias: the 4-wave transposed-read kernel, or with TTD_G4T=0 the
8-wave kernel + fold passes) against torch.mm (hipBLASLt, fp32 out, no bias sums).
usage: g4t_bench.py [--tokens T] [--wgs W] [--rounds R]"""
import sys

import torch

sys.path.insert(0, ".")
from tensorflow_train_distributed_amd.ops import gemm as G  # noqa: E402


def arg(name, default):
    return sys.argv[sys.argv.index(name) + 1] if name in sys.argv else default


T = int(arg("--tokens", "65536"))
WGS = int(arg("--wgs", "256"))
ROUNDS = int(arg("--rounds", "3"))
SHAPES = [("qkv", 3072, 1024), ("ao", 1024, 1024), ("ffn1", 4096, 1024), ("ffn2", 1024, 4096)]


def timeit(fn, iters=10):
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
    for name, M, N in SHAPES:
        dy = (torch.rand((T, M), device="cuda") * 2 - 1).bfloat16()
        x = (torch.rand((T, N), device="cuda") * 2 - 1).bfloat16()
        out = torch.empty(M, N, device="cuda")
        bias = torch.empty(M, device="cuda")
        splits = G.gemm_wgrad_splits(M, N, T, big_wgs=WGS)
        arms = {"engine": lambda: G.gemm_wgrad_bias(dy, x, out, bias, splits=splits),
                "torch": lambda: torch.mm(dy.t(), x, out_dtype=torch.float32, out=out)}
        res = {k: [] for k in arms}
        for _ in range(ROUNDS):
            for k, f in arms.items():
                res[k].append(timeit(f))
        fl = 2.0 * M * N * T
        line = "%-5s %5d x %5d x %6d splits %2d" % (name, M, N, T, splits)
        for k in arms:
            ms = min(res[k])
            line += "  %s %7.1f us %6.0f TF/s" % (k, ms * 1e3, fl / ms / 1e9)
        print(line, flush=True)


if __name__ == "__main__":
    main()
