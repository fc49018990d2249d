#!/usr/bin/env python3
"""LayerNorm backward only (BERT-Large b128 shape, dx with hidden dropout), repeated: rocprofv3
--pmc target. usage: python tools/ln_bwd_only.py [iters]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from tensorflow_train_distributed_amd.ops import transformer as T
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    dev = torch.device("cuda", 0)
    R, H = 65536, 1024
    x = torch.randn(R, H, device=dev).bfloat16()
    gamma = torch.rand(H, device=dev) + 0.5
    beta = torch.randn(H, device=dev)
    rng = T.RngState(7, dev)
    y, s, mean, rstd = T.layernorm_fwd(x, gamma, beta, rng=rng)
    dy = torch.randn(R, H, device=dev).bfloat16()
    dg = torch.zeros(H, device=dev)
    db = torch.zeros(H, device=dev)
    work = T.ln_bwd_workspace(R, H, dev)
    ds = torch.empty_like(dy)
    dx = torch.empty_like(dy)
    for _ in range(iters):
        T.layernorm_bwd(dy, s, mean, rstd, gamma, dg, db, ds_out=ds, want_dx=True, p_in=0.1, site_in=3, rng=rng,
                        work=work, dx_out=dx)
    torch.cuda.synchronize()
    print("done")


if __name__ == "__main__":
    main()
