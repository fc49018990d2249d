#!/usr/bin/env python3
"""Run one halo 3x3 conv variant (conv3_halo.hip) n times on the ResNet-50 stage-2 b1024 shape
(for rocprofv3 PMC passes). usage: one_c3.py {fwd|fwdbn|dgrad} [n]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from tensorflow_train_distributed_amd.ops import gemm as G  # noqa: E402
from tensorflow_train_distributed_amd.ops import kernels as K  # noqa: E402

mode, n = sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 10
B, H, W, C, N = 1024, 56, 56, 64, 64
M = B * H * W
x = torch.randn(B, H, W, C, device="cuda").bfloat16()
w = (torch.randn(N, 3, 3, C, device="cuda") / 24).bfloat16()
sc, sh = torch.rand(C, device="cuda") + 0.5, torch.randn(C, device="cuda") * 0.1
side = torch.empty_like(x)
sm = torch.empty(M * C // 8, dtype=torch.uint8, device="cuda")
y = torch.randn(B, H, W, N, device="cuda").bfloat16()
coef = torch.randn(3, N, device="cuda") * 0.1
fm = torch.randint(0, 256, (M * C // 8,), dtype=torch.uint8, device="cuda")
wt = K.krsc_to_crsk(w)
for _ in range(n):
    if mode == "fwd":
        G.conv3_halo(x, w, stat=True)
    elif mode == "fwdbn":
        G.conv3_halo(x, w, prologue=("bn_fwd", sc, sh, side, sm), stat=True)
    else:
        G.conv3_halo(x, wt, flip=True, prologue=("bn_bwd", y, None, coef, side), bn_stat=(y, fm))
torch.cuda.synchronize()
print("ok")
