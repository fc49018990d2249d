#!/usr/bin/env python3
"""Stem (7x7/s2, 3->64 channels padded to 8) weight-gradient sweep over tile and split-K at
ResNet-50 b1024: the kernel that ends every backward pass on the critical path.
usage: python tools/stem_wgrad_sweep.py [batch]"""
import sys

import torch

sys.path.insert(0, ".")
from tensorflow_train_distributed_amd.ops import gemm as G  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
x = torch.randn(B, 224, 224, 8, device="cuda").bfloat16()
dy = torch.randn(B, 112, 112, 64, device="cuda").bfloat16()
wshape = (64, 7, 7, 8)
g = G.conv_geom(x.shape, wshape, (2, 2), (3, 3))
base = G.wgrad_splits(g)
ref = G.conv_wgrad(x, dy, wshape, (2, 2), (3, 3))
fl = 2.0 * 64 * 392 * B * 112 * 112
for tile in ((64, 128), (64, 64), (128, 128), (128, 64)):
    for sp in (base // 2, base, base * 2):
        if sp < 1:
            continue
        f = lambda: G.conv_wgrad(x, dy, wshape, (2, 2), (3, 3), splits=sp, tile=tile)
        out = f()
        err = float((out - ref).abs().max() / ref.abs().max())
        for _ in range(2):
            f()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(5):
            f()
        e.record()
        torch.cuda.synchronize()
        t = s.elapsed_time(e) / 5 * 1e3
        print("tile %-10s splits %4d: %7.1f us %5.0f TF/s  (rel err vs default %.1e)" % (tile, sp, t, fl / t / 1e6, err),
              flush=True)
