#!/usr/bin/env python3
"""Does an engine path switch change one ResNet-50 training step beyond rounding? Same weights,
same batch: one forward+backward with the switch off, one with it on, one more off (the engine
is deterministic: off/off must match bit for bit). Reports the loss, the global gradient
difference and the worst variables. The switch is a ResNet attribute (e.g. pw_wgrad, bn_pro).
usage: python tools/grad_path_check.py --attr pw_wgrad [--batch 1024]"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--attr", required=True)
    ap.add_argument("--batch", type=int, default=1024)
    args = ap.parse_args()
    from tensorflow_train_distributed_amd.models.resnet import resnet50
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    B = args.batch
    m = resnet50(device=dev, seed=1234)
    g = torch.Generator(device=dev)
    g.manual_seed(0)
    x = torch.randn((B, 224, 224, 3), generator=g, device=dev).to(torch.bfloat16)
    y = torch.randint(0, 1000, (B,), generator=g, device=dev, dtype=torch.int32)
    P = m.params
    runs = {}
    for tag, on in (("off", False), ("on", True), ("off2", False)):
        setattr(m, args.attr, on)
        s = m.forward_backward(x, y, grad_scale=1.0 / B)
        torch.cuda.synchronize()
        runs[tag] = (float(s[0]), P.grad.clone())
    g0, g1, g2 = runs["off"][1], runs["on"][1], runs["off2"][1]
    rel = lambda a, b: float((a - b).norm() / (b.norm() + 1e-30))  # noqa: E731
    worst = []
    for sp in P.specs:
        if not sp.trainable:
            continue
        o, n = P.offsets[sp.name], P.var[sp.name].numel()
        worst.append((rel(g1[o:o + n], g0[o:o + n]), sp.name))
    worst.sort(reverse=True)
    out = {"attr": args.attr, "batch": B, "loss_off": runs["off"][0], "loss_on": runs["on"][0],
           "loss_off2": runs["off2"][0], "off_vs_off2_bitwise": bool(torch.equal(g0, g2)),
           "rel_grad_on_vs_off": rel(g1, g0), "cos_on_vs_off": float(torch.dot(g1, g0) / (g1.norm() * g0.norm())),
           "worst_vars": [(round(r, 7), nm) for r, nm in worst[:12]]}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
