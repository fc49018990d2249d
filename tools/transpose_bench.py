#!/usr/bin/env python3
"""Time the bf16 weight transpose (ops.kernels.krsc_to_crsk) at the BERT-Large weight shapes."""
import sys, torch
sys.path.insert(0, ".")
from tensorflow_train_distributed_amd.ops import kernels as K
for A, C in ((4096, 1024), (1024, 4096), (3072, 1024), (1024, 1024)):
    w = torch.randn(A, 1, 1, C, device="cuda").bfloat16()
    out = torch.empty(C, 1, 1, A, device="cuda", dtype=torch.bfloat16)
    for _ in range(3): K.krsc_to_crsk(w, out=out)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(50): K.krsc_to_crsk(w, out=out)
    e.record(); torch.cuda.synchronize()
    us = s.elapsed_time(e) / 50 * 1e3
    print("transpose %d x %d: %.1f us  %.2f TB/s" % (A, C, us, 2 * A * C * 2 / us / 1e6))
