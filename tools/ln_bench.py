#!/usr/bin/env python3
"""Standalone LayerNorm forward / backward at BERT-Large b128 (65536 x 1024 bf16): time per call
and HBM bandwidth (bytes the kernel must move / time), as the BERT step calls them (backward:
ds + dropout-masked dx out, hidden dropout 0.1).
usage: python tools/ln_bench.py [--rows 65536] [--hidden 1024]"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timed(fn, iters=20):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3  # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=65536)
    ap.add_argument("--hidden", type=int, default=1024)
    args = ap.parse_args()
    from tensorflow_train_distributed_amd.ops import transformer as T
    dev = torch.device("cuda", 0)
    R, H = args.rows, args.hidden
    x = torch.randn(R, H, device=dev).bfloat16()
    res = torch.randn(R, H, device=dev).bfloat16()
    gamma = torch.rand(H, device=dev) + 0.5
    beta = torch.randn(H, device=dev)
    rng = T.RngState(7, dev)
    y, s, mean, rstd = T.layernorm_fwd(x, gamma, beta, res=res, p_in=0.1, site_in=3, rng=rng)
    dy = torch.randn(R, H, device=dev).bfloat16()
    dg = torch.zeros(H, device=dev)
    db = torch.zeros(H, device=dev)
    work = T.ln_bwd_workspace(R, H, dev)
    ds = torch.empty_like(dy)
    dx = torch.empty_like(dy)
    el = R * H * 2
    out = {}
    t = timed(lambda: T.layernorm_fwd(x, gamma, beta, res=res, p_in=0.1, site_in=3, rng=rng, out=y, s_out=s,
                                      mean=mean, rstd=rstd))
    out["ln_fwd_res_drop_us"] = round(t, 1)
    out["ln_fwd_TBps"] = round(4 * el / t / 1e6, 2)  # x, res in; s, y out
    t = timed(lambda: T.layernorm_bwd(dy, s, mean, rstd, gamma, dg, db, ds_out=ds, want_dx=True, p_in=0.1,
                                      site_in=3, rng=rng, work=work, dx_out=dx))
    out["ln_bwd_dx_drop_us"] = round(t, 1)
    out["ln_bwd_TBps"] = round(4 * el / t / 1e6, 2)  # dy, s in; ds, dx out
    t = timed(lambda: T.layernorm_bwd(dy, s, mean, rstd, gamma, dg, db, ds_out=ds, work=work))
    out["ln_bwd_plain_us"] = round(t, 1)
    out["ln_bwd_plain_TBps"] = round(3 * el / t / 1e6, 2)
    # correctness vs fp32 autograd of the same LayerNorm (no dropout path)
    sf = s.float().requires_grad_(True)
    ref = torch.nn.functional.layer_norm(sf, (H,), gamma, beta, eps=1e-12)
    ref.backward(dy.float())
    T.layernorm_bwd(dy, s, mean, rstd, gamma, dg, db, ds_out=ds, work=work)
    out["ds_rel_err"] = float((ds.float() - sf.grad).norm() / sf.grad.norm())
    print(json.dumps(out))


if __name__ == "__main__":
    main()
