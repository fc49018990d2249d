"""Build + run the fp8 MFMA probe (on the GPU box): prints D for all-ones operands with
immediate and register scales, and for the non-scaled 16x16x32 instruction."""
import ctypes
import os
import subprocess
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
here = os.path.dirname(os.path.abspath(__file__))
so = os.path.join("/tmp", "libmfma_probe.so")
subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O2", "-shared", "-fPIC",
                       os.path.join(here, "mfma_fp8_probe.hip"), "-o", so])
lib = ctypes.CDLL(so)
ONE = 0x38  # e4m3 1.0
a = torch.full((64, 32), ONE, dtype=torch.uint8, device="cuda")
b = torch.full((64, 32), ONE, dtype=torch.uint8, device="cuda")
d = torch.zeros(64, 4, device="cuda")
for which, sa, sb in [(0, 127, 127), (1, 127, 127), (1, 0x7F7F7F7F, 0x7F7F7F7F), (2, 0, 0)]:
    d.zero_()
    rc = lib.probe(ctypes.c_void_p(a.data_ptr()), ctypes.c_void_p(b.data_ptr()), ctypes.c_void_p(d.data_ptr()),
                   sa, sb, which)
    print("which", which, "sa", hex(sa), "rc", rc, "D[0]", d[0].tolist(), "D[63]", d[63].tolist(), flush=True)
# k-mapping consistency: random codes, compare scaled mfma result vs numpy with lane map guess
from tensorflow_train_distributed_amd.ops import kernels as K
x = torch.randn(16, 128, device="cuda")
y = torch.randn(16, 128, device="cuda")
sc = torch.ones(1, device="cuda")
xq = K.quant_fp8(x.bfloat16(), sc)
yq = K.quant_fp8(y.bfloat16(), sc)
xd = K.dequant_fp8(xq, sc).float()
yd = K.dequant_fp8(yq, sc).float()
ref = xd @ yd.t()  # D[i][j] = sum_k X[i][k] Y[j][k]
for name, kmap in [("contig32", lambda g, j: 32 * g + j), ("split16", lambda g, j: (16 * g + j) if j < 16 else (64 + 16 * g + j - 16))]:
    A = torch.zeros(64, 32, dtype=torch.uint8, device="cuda")
    B = torch.zeros(64, 32, dtype=torch.uint8, device="cuda")
    for l in range(64):
        g = l >> 4
        for j in range(32):
            A[l, j] = xq[l & 15, kmap(g, j)]
            B[l, j] = yq[l & 15, kmap(g, j)]
    d.zero_()
    # D = A_op x B_op with A rows on lane&15 -> D[row][col] lane l holds col = l&15? rows 4g+i
    lib.probe(ctypes.c_void_p(B.data_ptr()), ctypes.c_void_p(A.data_ptr()), ctypes.c_void_p(d.data_ptr()), 127, 127, 0)
    got = torch.zeros(16, 16, device="cuda")
    for l in range(64):
        for i in range(4):
            got[l & 15, 4 * (l >> 4) + i] = d[l, i]  # swapped: row = X index on lane&15
    print(name, "max err", float((got - ref).abs().max()), "ref max", float(ref.abs().max()), flush=True)

# framework fp8 GEMM on all-ones and on random data
from tensorflow_train_distributed_amd.ops import gemm as G
a8 = torch.full((256, 256), ONE, dtype=torch.uint8, device="cuda")
b8 = torch.full((256, 256), ONE, dtype=torch.uint8, device="cuda")
y = G.gemm_fp8(a8, b8, out_dtype=torch.float32)
print("gemm_fp8 ones: expect 256 ->", float(y.min()), float(y.max()), flush=True)
print("quant codes for 1.0:", K.quant_fp8(torch.ones(8, device="cuda").bfloat16(), sc).tolist(), flush=True)
