#!/usr/bin/env python3
"""One-GPU interference harness for the N-rank co-scheduling policy (parallel/rccl.py).

At N > 1 the gradient buckets' RCCL kernels run on the communicator stream during the backward
and hold CUs; the backward's persistent kernels (one workgroup per CU, static work split) then
wait for those CUs. On one GPU this emulates it: the ResNet-50 step runs with its real
BucketedAllReducer, whose communicator is replaced by an emulator that launches, at every real
bucket point, a kernel of the communicator's CTA count on a normal-priority stream that streams
over a scratch buffer for as long as the bucket's ring all-reduce would take at --busbw GB/s
(plus --skew-us of waiting for the slowest peer). Modes:

  none      no emulated collectives (the one-GPU step)
  full      emulated collectives, persistent grids on every CU (no reservation)
  reserved  emulated collectives, persistent grids leave the CTA budget's CUs free (the policy)

usage: python tools/comm_interference.py [--batch 1024] [--ctas 8] [--busbw 150] [--world 8]
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


class EmulatedComm:
    def __init__(self, ctas, busbw_gbps, world, skew_us, device):
        from tensorflow_train_distributed_amd.parallel import rccl
        self.rccl = rccl
        self.max_ctas = ctas
        self.busbw = busbw_gbps
        self.world = world
        self.skew_us = skew_us
        self.stream = torch.cuda.Stream(device=device)  # normal priority, like the communicator's
        self.scratch = torch.zeros(64 << 20, dtype=torch.uint8, device=device)
        self.busy_us = 0.0

    def bucket(self, t, **kw):
        ev = torch.cuda.Event()
        ev.record()
        self.stream.wait_event(ev)
        nbytes = t.numel() * t.element_size()
        us = nbytes * 2.0 * (self.world - 1) / self.world / (self.busbw * 1e3) + self.skew_us
        self.busy_us += us
        self.rccl.emulate_bucket(self.stream, self.max_ctas, us, self.scratch)

    def join(self):
        torch.cuda.current_stream().wait_stream(self.stream)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--ctas", type=int, default=8)
    ap.add_argument("--busbw", type=float, default=150.0, help="emulated RCCL bus bandwidth, GB/s")
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--skew-us", type=float, default=200.0, help="per-bucket wait for the slowest peer")
    ap.add_argument("--modes", default="none,full,reserved,none,full,reserved")
    ap.add_argument("--out", default=None)
    args = ap.parse_args()

    from tensorflow_train_distributed_amd.models.resnet import resnet50
    from tensorflow_train_distributed_amd.parallel.collective import BucketedAllReducer
    from tensorflow_train_distributed_amd.train.flat import FlatSGD, Schedule
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    B = args.batch
    model = resnet50(device=dev, seed=1234)
    opt = FlatSGD(model.params, Schedule(kind=2, base_lr=0.1 * B / 256, warmup_steps=5, end_lr=0.0, power=2.0,
                                         total_steps=10000), momentum=0.9, weight_decay=5e-5)
    red = BucketedAllReducer(model.params)
    emu = EmulatedComm(args.ctas, args.busbw, args.world, args.skew_us, dev)
    g = torch.Generator(device=dev)
    g.manual_seed(0)
    images = torch.randn((B, 224, 224, 3), generator=g, device=dev).to(torch.bfloat16)
    labels = torch.randint(0, 1000, (B,), generator=g, device=dev, dtype=torch.int32)
    prio = torch.cuda.Stream(device=dev, priority=torch.cuda.Stream.priority_range()[1])
    prio.wait_stream(torch.cuda.current_stream())

    def step():
        with torch.cuda.stream(prio):
            red.begin()
            s = model.forward_backward(images, labels, grad_scale=1.0 / B, grad_hook=red.mark_ready)
            red.finish()
            opt.step()
            return s

    results = []
    for mode in args.modes.split(","):
        red.comm = None if mode == "none" else emu
        red.reserved_cus = args.ctas if mode == "reserved" else 0
        for _ in range(args.warmup):
            step()
        torch.cuda.synchronize()
        emu.busy_us = 0.0
        t0 = time.perf_counter()
        for _ in range(args.steps):
            step()
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / args.steps * 1e3
        r = {"mode": mode, "ms_per_step": round(ms, 3), "emulated_comm_ms_per_step": round(emu.busy_us / 1e3 / args.steps, 3),
             "buckets": len(red.buckets), "persistent_cus_in_backward": 256 - red.reserved_cus}
        results.append(r)
        print(json.dumps(r), flush=True)
    base = min(r["ms_per_step"] for r in results if r["mode"] == "none")
    summary = {"ctas": args.ctas, "busbw_GBps": args.busbw, "world": args.world, "skew_us": args.skew_us,
               "batch": B, "none_ms": base}
    for mode in ("full", "reserved"):
        v = [r["ms_per_step"] for r in results if r["mode"] == mode]
        if v:
            summary[mode + "_ms"] = min(v)
            summary[mode + "_loss_pct"] = round(100.0 * (min(v) - base) / base, 2)
    print(json.dumps(summary), flush=True)
    if args.out:
        with open(args.out, "w") as f:
            json.dump({"runs": results, "summary": summary}, f, indent=1)


if __name__ == "__main__":
    main()
