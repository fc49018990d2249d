#!/usr/bin/env python3
"""Run one ResNet conv GEMM repeatedly (for rocprofv3 --pmc passes).
usage: one_conv.py <layer from conv_bench.LAYERS> <fwd|dgrad|wgrad> [iters] [bm bn]"""
import sys

import torch

sys.path.insert(0, ".")
from tensorflow_train_distributed_amd.ops import gemm as G  # noqa: E402
from tools.conv_bench import LAYERS  # noqa: E402

name, op = sys.argv[1], sys.argv[2]
iters = int(sys.argv[3]) if len(sys.argv) > 3 else 20
tile = (int(sys.argv[4]), int(sys.argv[5])) if len(sys.argv) > 5 else (0, 0)
_, N, H, W, C, K, R, s, p = next(l for l in LAYERS if l[0] == name)
x = torch.randn(N, H, W, C, device="cuda").bfloat16()
w = (torch.randn(K, R, R, C, device="cuda") / (R * R * C) ** 0.5).bfloat16()
y = G.conv_fwd(x, w, (s, s), (p, p))
dy = torch.randn_like(y)
wt = w.permute(3, 1, 2, 0).contiguous()
for _ in range(iters):
    if op == "fwd":
        G.conv_fwd(x, w, (s, s), (p, p), tile=tile)
    elif op == "dgrad":
        G.conv_dgrad(dy, wt, x.shape, (s, s), (p, p), tile=tile)
    else:
        G.conv_wgrad(x, dy, w.shape, (s, s), (p, p), tile=tile)
torch.cuda.synchronize()
print("done")
