#!/usr/bin/env python3
"""Per-launch device time of one ResNet-50 (or BERT) training step, single HIP stream, every
native launch bracketed by HIP events (TTD_OP_TIMING=1) and GEMMs labelled with their shape.
Prints each launch in order with TF/s and the HBM/MFMA floor, then totals per launcher.

  TTD_WGRAD_STREAM=0 TTD_OP_TIMING=1 TTD_GEMM_LOG=1 python tools/op_timing.py [--batch 1024] [--model bert]
"""
import argparse
import os
import sys
from collections import defaultdict

os.environ.setdefault("TTD_OP_TIMING", "1")
os.environ.setdefault("TTD_GEMM_LOG", "1")
os.environ.setdefault("TTD_WGRAD_STREAM", "0")
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from tools.gemm_shapes_profile import _bytes  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--model", default="resnet50")
    ap.add_argument("--out", default="gpurun_out/op_timing.txt")
    args = ap.parse_args()
    from tensorflow_train_distributed_amd.ops import _lib
    dev = torch.device("cuda")
    if args.model == "resnet50":
        from tensorflow_train_distributed_amd.models.resnet import resnet50
        from tensorflow_train_distributed_amd.train.flat import FlatSGD, Schedule
        m = resnet50(device=dev)
        opt = FlatSGD(m.params, Schedule(kind=0, base_lr=0.01), momentum=0.9, weight_decay=5e-5)
        x = torch.randn(args.batch, 224, 224, 3, device=dev).bfloat16()
        y = torch.randint(0, 1000, (args.batch,), device=dev, dtype=torch.int32)

        def step():
            m.forward_backward(x, y)
            opt.step()
    else:
        from tensorflow_train_distributed_amd.models.bert import BertConfig, BertPretraining, synthetic_batch
        from tensorflow_train_distributed_amd.train.flat import FlatLAMB, Schedule
        cfg = BertConfig.large()
        m = BertPretraining(cfg, device=dev, seed=1)
        opt = FlatLAMB(m.params, Schedule(kind=0, base_lr=1e-4), weight_decay=0.01)
        b = synthetic_batch(cfg, args.batch, 512, max_predictions=80, device=dev, seed=0)

        def step():
            m.forward_backward(b)
            opt.step()
    for _ in range(2):
        step()
    torch.cuda.synchronize()
    _lib.TIMING.clear()
    t0 = torch.cuda.Event(enable_timing=True)
    t1 = torch.cuda.Event(enable_timing=True)
    t0.record()
    step()
    t1.record()
    torch.cuda.synchronize()
    lines = []
    tot = floor_tot = 0.0
    per = defaultdict(lambda: [0, 0.0, 0.0])
    for name, labels, s, e in _lib.TIMING:
        us = s.elapsed_time(e) * 1e3
        tot += us
        lab = ""
        fb = 0.0
        if labels:
            fl = sum(2.0 * M * N * K for _, M, N, K in labels)
            b = sum(_bytes(k, M, N, K) for k, M, N, K in labels)
            fb = max(b / 6.0e6, fl / 1.6e9)
            k0, M, N, K = labels[0]
            lab = "%-22s M=%-8d N=%-5d K=%-8d %5.0f TF/s %5.2f TB/s floor %7.1f" % (
                k0 + ("+%d" % (len(labels) - 1) if len(labels) > 1 else ""), M, N, K, fl / us / 1e6, b / us / 1e6, fb)
        floor_tot += fb
        key = name + (":" + labels[0][0].split("_")[0] if labels else "")
        per[key][0] += 1
        per[key][1] += us
        per[key][2] += fb
        lines.append("%9.1f us  %-28s %s" % (us, name.replace("ttdk_", ""), lab))
    lines.append("step wall %.1f us, launches %.1f us (sum), GEMM floor %.1f us" % (
        t0.elapsed_time(t1) * 1e3, tot, floor_tot))
    for k, (n, us, fb) in sorted(per.items(), key=lambda kv: -kv[1][1]):
        lines.append("  %-36s n=%4d %10.1f us  floor %9.1f" % (k, n, us, fb))
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    open(args.out, "w").write("\n".join(lines) + "\n")
    print("\n".join(lines[-30:]))


if __name__ == "__main__":
    main()
