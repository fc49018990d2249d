#!/usr/bin/env python3
"""Diagnose a segmented-capture replay mismatch on the small ResNet: replay normally and with a
device synchronize after every segment, against the eager steps (same seeds)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tensorflow_train_distributed_amd.models.resnet import ResNet  # noqa: E402
from tensorflow_train_distributed_amd.train.flat import FlatSGD, Schedule  # noqa: E402
from tensorflow_train_distributed_amd.utils import graphs  # noqa: E402


def make():
    m = ResNet(((64, 1, 1), (128, 2, 2)), num_classes=10, device="cuda", seed=5)
    o = FlatSGD(m.params, Schedule(kind=2, base_lr=0.1, warmup_steps=2, end_lr=0.0, power=2.0, total_steps=100),
                momentum=0.9, weight_decay=5e-5)
    return m, o


def main():
    torch.manual_seed(0)
    x = torch.randn(16, 32, 32, 3, device="cuda").bfloat16()
    y = torch.randint(0, 10, (16,), device="cuda", dtype=torch.int32)

    def step(m, o):
        s = m.forward_backward(x, y)
        o.step()
        return s

    m1, o1 = make()
    eager = [step(m1, o1).clone() for _ in range(3)]
    res = {"eager": [[round(float(v), 5) for v in e] for e in eager], "env": {k: v for k, v in os.environ.items() if k.startswith("TTD_")}}
    for serial in (False, True):
        m2, o2 = make()
        main_s = torch.cuda.Stream(priority=torch.cuda.Stream.priority_range()[1])
        seg = graphs.capture_segmented(lambda: step(m2, o2), main=main_s, warmup=1)
        outs = []
        for _ in range(2):
            if serial:
                for s, g in seg.cap.segments:
                    with torch.cuda.stream(s):
                        g.replay()
                    torch.cuda.synchronize()
                r = seg.outputs
            else:
                r = seg.replay()
            torch.cuda.synchronize()
            outs.append([round(float(v), 5) for v in r])
        res["serial" if serial else "replay"] = outs
        res["info"] = seg.info
        res["order"] = ["main" if s is main_s else "side" for s, _ in seg.cap.segments]
    print(json.dumps(res))


if __name__ == "__main__":
    main()
