#!/usr/bin/env python3
"""Per-workgroup clock stamps of the dK/dV attention backward kernel (attn_bwd_kv_kernel MODE bit 3,
TTD_ATTN_KV_DIAG=8 | other bits): median prologue / tile loop / epilogue cycles, workgroup
lifetime, and the kernel span from the 100 MHz real-time clock, at BERT-Large b128 with dropout.
usage: TTD_ATTN_KV_DIAG=8 python tools/attn_kv_stamps.py [B]"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from tensorflow_train_distributed_amd.ops import transformer as T  # noqa: E402

assert int(os.environ.get("TTD_ATTN_KV_DIAG", "0")) & 8, "set TTD_ATTN_KV_DIAG with bit 3"
B, H, S, D = (int(sys.argv[1]) if len(sys.argv) > 1 else 128), 16, 512, 64
qkv = (torch.randn(B * S, 3 * H * D, device="cuda") * 0.5).bfloat16()
q, k, v = qkv[:, :H * D], qkv[:, H * D:2 * H * D], qkv[:, 2 * H * D:]
out = torch.empty(B * S, H * D, device="cuda", dtype=torch.bfloat16)
lse = torch.empty(B * H, S, device="cuda")
dout = torch.randn_like(out)
rng = T.RngState(7, "cuda")
T.attention_fwd(q, k, v, out, lse, B, H, S, p_drop=0.1, rng=rng)
nwg = B * H * (S // 128)
dv = torch.zeros(max(B * S * H * D, nwg * 32), device="cuda", dtype=torch.bfloat16)  # >= nwg * 64 B
dq = torch.empty_like(out)
dk = torch.empty_like(out)
for _ in range(4):  # warm clocks
    T.attention_bwd(q, k, v, out, dout, lse, dq, dk, dv[:B * S * H * D].view(B * S, H * D), B, H, S, p_drop=0.1, rng=rng)
torch.cuda.synchronize()
st = dv.view(torch.int64)[:nwg * 8].view(nwg, 8).cpu().numpy()
pro, loop, epi = st[:, 1] - st[:, 0], st[:, 2] - st[:, 1], st[:, 3] - st[:, 2]
life = st[:, 3] - st[:, 0]
real = st[:, 5] - st[:, 4]
span = (st[:, 5].max() - st[:, 4].min()) / 100.0  # us
clk = np.median(life / np.maximum(real, 1)) * 100.0  # MHz
print("workgroups %d  kernel span %.1f us  clock ~%.0f MHz" % (nwg, span, clk))
for name, x in (("prologue", pro), ("tile loop", loop), ("epilogue", epi), ("lifetime", life)):
    print("  %-10s median %8.0f  p10 %8.0f  p90 %8.0f cycles" % (name, np.median(x), np.percentile(x, 10), np.percentile(x, 90)))
# concurrency: workgroups resident per CU id over time
t0 = st[:, 4].min()
print("  mean resident workgroups: %.1f (sum of lifetimes / span)" % (real.sum() / 100.0 / span))
cus = st[:, 7]
print("  distinct CU ids %d" % len(np.unique(cus)))
