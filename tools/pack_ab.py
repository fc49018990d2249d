#!/usr/bin/env python3
"""A/B of two builds of libttd_hip on the bench's ResNet-50 step (TTD_HIP_LIB_OVERRIDE picks the
build): per-step losses and, after step 1, every variable's gradient, saved to /tmp for
`--compare`. Used to locate where two builds that should agree bitwise first differ.

    python tools/pack_ab.py --tag new --steps 3
    TTD_HIP_LIB_OVERRIDE=.../libttd_hip_oldpack.so python tools/pack_ab.py --tag old --steps 3
    python tools/pack_ab.py --compare new old
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run(args):
    from tensorflow_train_distributed_amd.models.resnet import resnet50
    from tensorflow_train_distributed_amd.train.flat import FlatSGD, Schedule
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    B = args.batch
    model = resnet50(device=dev, seed=1234)
    opt = FlatSGD(model.params, Schedule(kind=2, base_lr=0.1 * B / 256, warmup_steps=5, end_lr=0.0, power=2.0,
                                         total_steps=10000), momentum=0.9, weight_decay=5e-5)
    g = torch.Generator(device=dev)
    g.manual_seed(0)
    images = torch.randn((B, 224, 224, 3), generator=g, device=dev).to(torch.bfloat16)
    labels = torch.randint(0, 1000, (B,), generator=g, device=dev, dtype=torch.int32)
    P = model.params
    out = {"loss": []}
    for s in range(args.steps):
        sums = model.forward_backward(images, labels, grad_scale=1.0 / B)
        torch.cuda.synchronize()
        out["loss"].append(float(sums[0]))
        if s == 0:
            out["grad"] = {n: P.g[n].detach().float().cpu().clone() for n in P.names()}
            out["order"] = list(P.names())
        opt.step()
    torch.save(out, "/tmp/pack_ab_%s.pt" % args.tag)
    print(args.tag, "losses", " ".join("%.9g" % v for v in out["loss"]), flush=True)


def compare(a, b):
    A = torch.load("/tmp/pack_ab_%s.pt" % a, weights_only=True)
    Bd = torch.load("/tmp/pack_ab_%s.pt" % b, weights_only=True)
    print("losses", a, A["loss"])
    print("losses", b, Bd["loss"])
    ndiff = 0
    for n in A["order"]:  # forward order; the backward reaches the head first
        x, y = A["grad"][n], Bd["grad"][n]
        if not torch.equal(x, y):
            ndiff += 1
            rel = float((x - y).norm() / max(float(y.norm()), 1e-30))
            nbits = int((x.view(torch.int32) != y.view(torch.int32)).sum())
            print("differs %-48s rel %.3e  elements %d / %d" % (n, rel, nbits, x.numel()))
    print("variables differing after step 1: %d / %d" % (ndiff, len(A["order"])))


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--tag", default="x")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--compare", nargs=2)
    a = ap.parse_args()
    if a.compare:
        compare(*a.compare)
    else:
        run(a)
