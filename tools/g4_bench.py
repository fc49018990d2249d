#!/usr/bin/env python3
"""Time the 4-wave AGPR GEMM (ops.gemm.gemm4w) against the 8-wave 256-row kernel
(ops.gemm.gemm, trans_b) and torch.matmul (hipBLASLt) on random bf16 operands, interleaved
rounds in one process. Prints TF/s per shape and arm.
usage: g4_bench.py [--tokens T] [--only SUBSTR] [--rounds R] [--arms g4,big,torch]"""
import sys

import torch

sys.path.insert(0, ".")
from tensorflow_train_distributed_amd.ops import gemm as G  # noqa: E402


def arg(name, default):
    return sys.argv[sys.argv.index(name) + 1] if name in sys.argv else default


T = int(arg("--tokens", "65536"))
ONLY = arg("--only", None)
ROUNDS = int(arg("--rounds", "3"))
ARMS = arg("--arms", "g4:3,g4:30,g4:0,big,torch").split(",")
SHAPES = [  # (name, M, N, K, epilogue)
    ("sq4096", 4096, 4096, 4096, ""),
    ("sq8192", 8192, 8192, 8192, ""),
    ("bert_qkv_fwd", T, 3072, 1024, "bias"),
    ("bert_ffn1_fwd", T, 4096, 1024, "gelu"),
    ("bert_ffn2_fwd", T, 1024, 4096, "bias"),
    ("bert_ao_fwd", T, 1024, 1024, "bias"),
    ("bert_ffn1_dgrad", T, 1024, 4096, ""),
    ("bert_ffn2_dgrad", T, 4096, 1024, "dgelu"),
    ("bert_mlm_logits", 10240, 30592, 1024, "bias"),
]


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
    for name, M, N, K, ep in SHAPES:
        if ONLY and ONLY not in name:
            continue
        a = (torch.rand((M, K), device="cuda") * 2 - 1).bfloat16()
        b = (torch.rand((N, K), device="cuda") * 2 - 1).bfloat16()
        bias = torch.randn(N, device="cuda") if ep in ("bias", "gelu") else None
        res = torch.randn(M, N, device="cuda").bfloat16() if ep == "dgelu" else None
        aux = torch.empty(M, N, device="cuda", dtype=torch.bfloat16) if ep == "gelu" else None
        act = {"gelu": G.ACT_GELU, "dgelu": G.ACT_DGELU}.get(ep, G.ACT_NONE)
        out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        b16 = bias.bfloat16() if bias is not None else None
        arms = {
            "big": lambda: G.gemm(a, b, trans_b=True, out=out, bias=bias, act=act, residual=res, aux=aux),
            "torch": (lambda: torch.addmm(b16, a, b.t(), out=out)) if b16 is not None
            else (lambda: torch.mm(a, b.t(), out=out)),
        }
        for k in ARMS:
            if k.startswith("g4:"):  # g4:SCHED[/GROUP[/STAGGER]]
                sv, _, rest = k[3:].partition("/")
                gv, _, stv = rest.partition("/")
                arms[k] = (lambda v, gr, sg: lambda: (G.set_g4_sched(v), G.set_g4_group(gr), G.set_g4_stagger(sg),
                                                      G.gemm4w(a, b, out=out, bias=bias, act=act, residual=res,
                                                               aux=aux)))(int(sv), int(gv or 8), int(stv or 1))
        fl = 2.0 * M * N * K
        res_t = {k: [] for k in ARMS}
        for _ in range(ROUNDS):
            for k in ARMS:
                res_t[k].append(timeit(arms[k]))
        line = "%-16s %6d x %5d x %5d %-5s" % (name, M, N, K, ep)
        for k in ARMS:
            ms = min(res_t[k])
            line += "  %s %7.1f us %6.0f TF/s" % (k, ms * 1e3, fl / ms / 1e9)
        print(line, flush=True)


if __name__ == "__main__":
    main()
