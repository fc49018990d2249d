#!/usr/bin/env python3
"""Wave-quantisation probe of the 256-row conv GEMM: TF/s of the stage-4/5 3x3 convs at batch
1024 vs batches whose tile count fills whole rounds of 256 workgroups."""
import sys

import torch

sys.path.insert(0, ".")
from tensorflow_train_distributed_amd.ops import gemm as G  # noqa: E402


def timeit(fn, iters=10):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


for (H, C, K), batches in (((14, 256, 256), (1024, 1306, 1337)), ((7, 512, 512), (1024, 1337, 1306)),
                           ((28, 128, 128), (1024, 1045))):
    for B in batches:
        x = torch.randn(B, H, H, C, device="cuda").bfloat16()
        w = (torch.randn(K, 3, 3, C, device="cuda") / (9 * C) ** 0.5).bfloat16()
        M = B * H * H
        fl = 2.0 * M * K * 9 * C
        line = "H=%2d C=%3d B=%4d M=%7d tiles256=%6.2f rounds" % (H, C, B, M, M / 256 * max(1, K // 256) / 256)
        for t in ((256, 256), (256, 128), (128, 128)):
            try:
                us = timeit(lambda: G.conv_fwd(x, w, (1, 1), (1, 1), tile=t))
                line += " | %s %6.1f us %5.0f TF/s" % (t, us, fl / us / 1e6)
            except Exception as ex:  # noqa: BLE001
                line += " | %s n/a" % (t,)
        print(line, flush=True)
