#!/usr/bin/env python3
"""Phase timing of the persistent 4-wave GEMM from in-kernel s_memtime stamps (diagnostic build
TTD_G4_SCHED=31): per tile, cycles from tile start to K-tile 0 landed, the main loop, the
epilogue. usage: g4_stamps.py M N K [epilogue: none|bias|gelu|dgelu]"""
import ctypes
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from tensorflow_train_distributed_amd.ops import _lib  # noqa: E402
from tensorflow_train_distributed_amd.ops import gemm as G  # noqa: E402

M, N, K = (int(x) for x in sys.argv[1:4])
ep = sys.argv[4] if len(sys.argv) > 4 else "none"
_lib.register({"ttdk_g4_stamps": [_lib.P]})
a = (torch.rand((M, K), device="cuda") * 2 - 1).bfloat16()
b = (torch.rand((N, K), device="cuda") * 2 - 1).bfloat16()
bias = torch.randn(N, device="cuda") if ep in ("bias", "gelu") else None
res = torch.randn(M, N, device="cuda").bfloat16() if ep == "dgelu" else None
aux = torch.empty(M, N, device="cuda", dtype=torch.bfloat16) if ep == "gelu" else None
act = {"gelu": G.ACT_GELU, "dgelu": G.ACT_DGELU}.get(ep, G.ACT_NONE)
out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
G.set_g4_sched(31)
for _ in range(3):
    G.gemm4w(a, b, out=out, bias=bias, act=act, residual=res, aux=aux)
torch.cuda.synchronize()
buf = np.zeros(2048 * 4 * 4, dtype=np.uint64)
_lib.call("ttdk_g4_stamps", buf.ctypes.data_as(ctypes.c_void_p))
st = buf.reshape(2048, 4, 4).astype(np.float64)
live = st[:, :, 3] > 0
n = st[:, :, 3][live]
for i, nm in enumerate(["land", "mainloop", "epilogue"]):
    v = st[:, :, i][live] / n
    print("%-9s per tile: mean %8.0f  min %8.0f  max %8.0f cycles" % (nm, v.mean(), v.min(), v.max()))
print("tiles per wave: mean %.1f; K-tiles %d -> main loop per K-tile %.0f cycles (ideal 2048)" % (
    n.mean(), K // 64, (st[:, :, 1][live] / n).mean() / (K // 64)))
