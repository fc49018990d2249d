#!/usr/bin/env python3
"""How far ahead of the GPU does the host run in the eager ResNet-50 step?

Times the Python issue of each step (host wall time of the call, no synchronisation) against
the GPU's own step time (events on the main stream), and the host lead at the start of each
backward: if the host issues about as fast as the GPU executes, eager steps throttle the
weight-gradient side stream (its kernels are queued just in time) in a way a hipGraph replay,
which queues the whole step at once, does not.

    python tools/host_issue_probe.py [--batch 1024] [--steps 10]
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--steps", type=int, default=10)
    a = ap.parse_args()
    from tensorflow_train_distributed_amd.models.resnet import resnet50
    from tensorflow_train_distributed_amd.train.flat import FlatSGD, Schedule
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    B = a.batch
    model = resnet50(device=dev, seed=1234)
    opt = FlatSGD(model.params, Schedule(kind=2, base_lr=0.1 * B / 256, warmup_steps=5, end_lr=0.0, power=2.0,
                                         total_steps=10000), momentum=0.9, weight_decay=5e-5)
    g = torch.Generator(device=dev)
    g.manual_seed(0)
    images = torch.randn((B, 224, 224, 3), generator=g, device=dev).to(torch.bfloat16)
    labels = torch.randint(0, 1000, (B,), generator=g, device=dev, dtype=torch.int32)
    prio = torch.cuda.Stream(device=dev, priority=torch.cuda.Stream.priority_range()[1])

    def step():
        model.forward_backward(images, labels, grad_scale=1.0 / B)
        opt.step()

    with torch.cuda.stream(prio):
        for _ in range(4):
            step()
    torch.cuda.synchronize()
    host, evs = [], []
    with torch.cuda.stream(prio):
        t_start = time.perf_counter()
        for _ in range(a.steps):
            e = torch.cuda.Event(enable_timing=True)
            e.record(prio)
            t0 = time.perf_counter()
            step()
            host.append((time.perf_counter() - t0) * 1e3)
            evs.append((e, time.perf_counter() - t_start))
        end = torch.cuda.Event(enable_timing=True)
        end.record(prio)
    t_issue_done = time.perf_counter() - t_start
    torch.cuda.synchronize()
    t_all = time.perf_counter() - t_start
    gpu = [evs[i][0].elapsed_time(evs[i + 1][0]) for i in range(len(evs) - 1)] + [evs[-1][0].elapsed_time(end)]
    res = {"host_issue_ms_per_step": [round(x, 2) for x in host], "gpu_ms_per_step": [round(x, 2) for x in gpu],
           "host_issue_total_s": round(t_issue_done, 3), "wall_total_s": round(t_all, 3)}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
